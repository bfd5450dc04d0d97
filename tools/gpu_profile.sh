# Round-1 evidence run: GPU parity tests, the C2 bench line, a rocprofv3
# kernel-trace summary of the same bench command, and FETCH/WRITE_SIZE passes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 300 python bench.py --steps 50 --warmup 5 > gpurun_out/bench_c2.log 2>&1 || { echo BENCH_FAILED; tail -20 gpurun_out/bench_c2.log; exit 1; }
tail -1 gpurun_out/bench_c2.log | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/kt -o kt --output-format csv -- python3 bench.py --steps 50 --warmup 5 --no-cpu > gpurun_out/prof/kt.log 2>&1 || { echo PROF_FAILED; tail -20 gpurun_out/prof/kt.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof/fetch -o f --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu > gpurun_out/prof/f.log 2>&1 || { echo PMC1_FAILED; tail -5 gpurun_out/prof/f.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof/write -o w --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu > gpurun_out/prof/w.log 2>&1 || { echo PMC2_FAILED; tail -5 gpurun_out/prof/w.log; exit 1; }
find gpurun_out/prof -name "*.csv" | head -20
timeout -k 10 300 python bench.py --config C5 --steps 20 --warmup 3 > gpurun_out/bench_c5.log 2>&1 || { echo C5_FAILED; tail -5 gpurun_out/bench_c5.log; exit 1; }
timeout -k 10 300 python bench.py --config C4 --budget 65536 --steps 3 --warmup 1 > gpurun_out/bench_c4.log 2>&1 || { echo C4_FAILED; tail -5 gpurun_out/bench_c4.log; exit 1; }
timeout -k 10 300 python bench.py --config C3 --keys 20000 --steps 5 --warmup 1 --no-cpu > gpurun_out/bench_c3s.log 2>&1 || { echo C3_FAILED; tail -5 gpurun_out/bench_c3s.log; exit 1; }
timeout -k 10 300 python bench.py --config C1 --steps 20 --warmup 3 > gpurun_out/bench_c1.log 2>&1 || { echo C1_FAILED; tail -5 gpurun_out/bench_c1.log; exit 1; }
tail -1 gpurun_out/bench_c1.log | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/kt4 -o kt4 --output-format csv -- python3 bench.py --config C4 --budget 65536 --steps 3 --warmup 1 --no-cpu > gpurun_out/prof/kt4.log 2>&1 || { echo PROF4_FAILED; tail -20 gpurun_out/prof/kt4.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof/fetch4 -o f4 --output-format csv -- python3 bench.py --config C4 --budget 65536 --steps 2 --warmup 1 --no-cpu > gpurun_out/prof/f4.log 2>&1 || { echo PMC41_FAILED; tail -5 gpurun_out/prof/f4.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof/write4 -o w4 --output-format csv -- python3 bench.py --config C4 --budget 65536 --steps 2 --warmup 1 --no-cpu > gpurun_out/prof/w4.log 2>&1 || { echo PMC42_FAILED; tail -5 gpurun_out/prof/w4.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_ATOMIC_sum -d gpurun_out/prof/atom4 -o a4 --output-format csv -- python3 bench.py --config C4 --budget 65536 --steps 2 --warmup 1 --no-cpu > gpurun_out/prof/a4.log 2>&1 || { echo PMC43_FAILED; tail -5 gpurun_out/prof/a4.log; exit 1; }
echo ALL_OK
