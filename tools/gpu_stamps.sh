# Phase stamps of k_spec (diagnostic build) on C2, raw arrays saved for offline fits.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/stamps
mkdir -p $O
export LINCHECK_LIB_OVERRIDE=$PWD/jepsen-etcd-demo_amd/lincheck/liblincheck_specst.so
for f in 0x100 0; do
  timeout -k 10 300 python -u tools/spec_stamps.py 1000 4 $f $O/st4_$f.npz > $O/st4_$f.txt 2>&1 || { tail -5 $O/st4_$f.txt; exit 1; }
done
timeout -k 10 300 python -u tools/spec_stamps.py 1000 8 0x100 $O/st8.npz > $O/st8.txt 2>&1 || { tail -5 $O/st8.txt; exit 1; }
head -12 $O/st8.txt
echo ALL_OK
