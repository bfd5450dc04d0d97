# Rerun-launch grid: cu_count x 1 workgroups against x 8 (C2 / C5 steps).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/rr
mkdir -p $O
timeout -k 10 200 python -u tools/spec_ab.py C2 1000 1000 default 2>&1 | tee $O/ab_c2.txt || exit 1
LINCHECK_LIB_OVERRIDE=$PWD/jepsen-etcd-demo_amd/lincheck/liblincheck_rr1.so timeout -k 10 200 python -u tools/spec_ab.py C2 1000 1000 default 2>&1 | tee -a $O/ab_c2.txt || exit 1
timeout -k 10 200 python -u tools/spec_ab.py C5 1000 1000 default 2>&1 | tee $O/ab_c5.txt || exit 1
LINCHECK_LIB_OVERRIDE=$PWD/jepsen-etcd-demo_amd/lincheck/liblincheck_rr1.so timeout -k 10 200 python -u tools/spec_ab.py C5 1000 1000 default 2>&1 | tee -a $O/ab_c5.txt || exit 1
echo ALL_OK
