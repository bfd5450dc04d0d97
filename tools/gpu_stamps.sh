# Phase stamps of k_spec (diagnostic build) on C2, raw arrays saved for offline fits.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/stamps
mkdir -p $O
export LINCHECK_LIB_OVERRIDE=$PWD/jepsen-etcd-demo_amd/lincheck/liblincheck_specst.so
timeout -k 10 300 python -u tools/spec_stamps.py 1000 4 0 $O/st4_r3.npz > $O/st4_r3.txt 2>&1 || { tail -5 $O/st4_r3.txt; exit 1; }
head -14 $O/st4_r3.txt
echo ALL_OK
