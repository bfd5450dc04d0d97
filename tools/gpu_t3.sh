# T3 (HBM tier) check: GPU parity suite, then C4 bench lines at two budgets.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 300 python bench.py --config C4 --budget 65536 --steps 3 --warmup 1 > gpurun_out/bench_c4.log 2>&1 || { echo C4_FAILED; tail -5 gpurun_out/bench_c4.log; exit 1; }
tail -1 gpurun_out/bench_c4.log | cut -c1-200
timeout -k 10 300 python bench.py --config C4 --budget 1048576 --steps 2 --warmup 1 --no-cpu > gpurun_out/bench_c4_b20.log 2>&1 || { echo C4B20_FAILED; tail -5 gpurun_out/bench_c4_b20.log; exit 1; }
tail -1 gpurun_out/bench_c4_b20.log | cut -c1-200
echo ALL_OK
