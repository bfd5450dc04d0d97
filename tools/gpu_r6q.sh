# Round 6: exact speculative segments (Jepsen-shaped calls) at 4 vs 8 per key.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6q; mkdir -p $O
timeout -k 10 400 python -u tools/ex_segs_ab.py > $O/ex.txt 2>&1 || { tail -10 $O/ex.txt; exit 1; }
cat $O/ex.txt
