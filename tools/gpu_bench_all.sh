# Bench lines for every config on one GPU (with CPU baselines), C4 at the default 2^20 budget too.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
run() { n=$1; shift; timeout -k 10 400 python -u bench.py "$@" > gpurun_out/bench_$n.log 2>&1 || { echo "$n FAILED"; tail -5 gpurun_out/bench_$n.log; exit 1; }; echo "$n $(tail -1 gpurun_out/bench_$n.log | cut -c1-160)"; }
run c2 --steps 50 --warmup 5
run c5 --config C5 --steps 20 --warmup 3
run c1 --config C1 --steps 20 --warmup 3
run c4 --config C4 --budget 65536 --steps 3 --warmup 1
run c4b20 --config C4 --steps 2 --warmup 1
echo ALL_OK
