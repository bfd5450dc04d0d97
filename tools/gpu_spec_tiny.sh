set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/tiny
mkdir -p $O
LINCHECK_LIB_OVERRIDE=$PWD/jepsen-etcd-demo_amd/lincheck/liblincheck_dbg.so timeout -k 10 40 python -u tools/spec_tiny.py 1 spec_segs=0x202 > $O/dbg.txt 2>&1 || { echo "FAILED"; head -40 $O/dbg.txt; exit 1; }
head -40 $O/dbg.txt
echo ALL_OK
