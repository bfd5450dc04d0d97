# Speculative segments on fewer waves (block-local queues): a bounded tiny
# check of each configuration first, then C2 / C5 at segments x waves 8x4
# (default), 4x4, 12x4, 16x4, 8x8; a C3 shard at 2x2 (default), 4x2, 8x2.
# Records compared across settings.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/specw
mkdir -p $O
for s in spec_segs=0x202 spec_segs=0x404 spec_segs=0x408 spec_segs=0x204 spec_segs=8; do
timeout -k 10 60 python -u tools/spec_tiny.py 64 $s 2>&1 | tee -a $O/tiny.txt || { echo "FAILED $s"; exit 1; }
done
timeout -k 10 200 python -u tools/spec_ab.py C2 1000 1000 default spec_segs=0x404 spec_segs=0x40c spec_segs=0x410 spec_segs=8 2>&1 | tee $O/ab_c2.txt || exit 1
timeout -k 10 200 python -u tools/spec_ab.py C5 1000 1000 default spec_segs=0x404 spec_segs=0x40c 2>&1 | tee $O/ab_c5.txt || exit 1
timeout -k 10 200 python -u tools/spec_ab.py C3 12500 2000 default spec_segs=0x204 spec_segs=0x208 2>&1 | tee $O/ab_c3s.txt || exit 1
echo ALL_OK
