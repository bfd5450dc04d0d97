# C3 at full size on one GPU (100,000 keys x 2,000 ops), plus the C1 line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 python bench.py --config C1 --steps 20 --warmup 3 > gpurun_out/bench_c1.log 2>&1 || { echo C1_FAILED; tail -5 gpurun_out/bench_c1.log; exit 1; }
tail -1 gpurun_out/bench_c1.log | cut -c1-250
timeout -k 10 600 python -u bench.py --config C3 --steps 5 --warmup 1 --no-cpu > gpurun_out/bench_c3.log 2>&1 || { echo C3_FAILED; tail -5 gpurun_out/bench_c3.log; exit 1; }
tail -1 gpurun_out/bench_c3.log | cut -c1-300
