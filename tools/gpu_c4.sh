# C4 bench lines (2^16 and 2^20 budgets) and the layered tier's GPU tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/c4
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_layers.py tests/test_abi.py -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|^E " $O/tests.log | head -20; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u bench.py --config C4 --budget 65536 --steps 5 --warmup 1 > $O/bench_c4.json 2> $O/bench_c4.err || { tail -5 $O/bench_c4.err; exit 1; }
cut -c1-200 $O/bench_c4.json
timeout -k 10 300 python -u bench.py --config C4 --budget 1048576 --steps 2 --warmup 1 --no-cpu > $O/bench_c4_b20.json 2> $O/bench_c4_b20.err || { tail -5 $O/bench_c4_b20.err; exit 1; }
echo ALL_OK
