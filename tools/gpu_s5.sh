# Five speculative segments per key (5-wave workgroups) against four, C2 / C5.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/s5
mkdir -p $O
export LINCHECK_LIB_OVERRIDE=$PWD/jepsen-etcd-demo_amd/lincheck/liblincheck_s5.so
timeout -k 10 200 python -u tools/spec_ab.py C2 1000 1000 default spec_segs=5 spec_segs=6 2>&1 | tee $O/ab_c2.txt || exit 1
timeout -k 10 200 python -u tools/spec_ab.py C5 1000 1000 default spec_segs=5 2>&1 | tee $O/ab_c5.txt || exit 1
echo ALL_OK
