# Round 6: segments per key on a C3 shard (12,500 x 2,000) with the
# overlapped build: 2 (default), 4 and 8.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6s; mkdir -p $O
timeout -k 10 300 python -u tools/spec_ab.py C3 12500 2000 default spec_segs=4 spec_segs=8 > $O/c3.txt 2>&1 || { tail -5 $O/c3.txt; exit 1; }
cat $O/c3.txt
