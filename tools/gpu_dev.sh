# Development call: one test file (arg 1) and a short bench run (C2 default).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest ${1:-tests/test_gpu_node.py} -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/dev_tests.log 2>&1
rc=$?
grep -E "FAILED|ERROR|^E " gpurun_out/dev_tests.log | head -30
tail -2 gpurun_out/dev_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 ${BENCH_ARGS:-} > gpurun_out/dev_bench.json 2> gpurun_out/dev_bench.err
rc=$?
tail -3 gpurun_out/dev_bench.err
cat gpurun_out/dev_bench.json
exit $rc
