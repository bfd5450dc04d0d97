# Per-key phase cycles of the layered HBM tier on C4 (LC_T3L_CNT build).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/t3cnt
mkdir -p $O
LINCHECK_LIB_OVERRIDE=$PWD/jepsen-etcd-demo_amd/lincheck/liblincheck_t3lcnt.so timeout -k 10 200 python -u tools/t3l_cnt.py 65536 256 2>&1 | tee $O/cnt.txt || exit 1
echo ALL_OK
