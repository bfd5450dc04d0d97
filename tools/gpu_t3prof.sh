set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 120 python -u tools/t3_prof.py 65536 > gpurun_out/t3_plain.log 2>&1 || { echo PLAIN_FAILED; tail -20 gpurun_out/t3_plain.log; exit 1; }
cat gpurun_out/t3_plain.log
LINCHECK_LIB_OVERRIDE=$GRAFT_REPO_ROOT/jepsen-etcd-demo_amd/lincheck/liblincheck_t3prof.so timeout -k 10 120 python -u tools/t3_prof.py 65536 > gpurun_out/t3_prof.log 2>&1 || { echo PROF_FAILED; tail -20 gpurun_out/t3_prof.log; exit 1; }
grep -c T3PROF gpurun_out/t3_prof.log
