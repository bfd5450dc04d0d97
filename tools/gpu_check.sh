set -o pipefail
cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/bench_c2.log 2>&1 || { echo BENCH_FAILED; tail -20 gpurun_out/bench_c2.log; exit 1; }
tail -1 gpurun_out/bench_c2.log
