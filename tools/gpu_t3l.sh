# Layered HBM tier: its GPU tests, the T3 tests of the other files, then C4
# at 2^16 with and without it, and a kernel-trace profile of the layered run.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/t3l
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_layers.py -x -v --timeout 200 --timeout-method thread > $O/tests_layers.log 2>&1 || { echo LAYER_TESTS_FAILED; grep -E "FAILED|^E |Error" $O/tests_layers.log | head -30; exit 1; }
tail -2 $O/tests_layers.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -v --timeout 200 --timeout-method thread -k "hbm or c4 or wide or counterexamples or window or many" > $O/tests_t3.log 2>&1 || { echo T3_TESTS_FAILED; grep -E "FAILED|^E |Error" $O/tests_t3.log | head -30; exit 1; }
tail -2 $O/tests_t3.log
timeout -k 10 300 python -u bench.py --config C4 --budget 65536 --steps 3 --warmup 1 --no-cpu > $O/bench_c4_layers.json 2> $O/bench_c4_layers.err || { tail -5 $O/bench_c4_layers.err; exit 1; }
cut -c1-300 $O/bench_c4_layers.json
LC_T3_LAYERS=0 timeout -k 10 300 python -u bench.py --config C4 --budget 65536 --steps 3 --warmup 1 --no-cpu > $O/bench_c4_old.json 2> $O/bench_c4_old.err || { tail -5 $O/bench_c4_old.err; exit 1; }
cut -c1-300 $O/bench_c4_old.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt_c4 -o kt4 --output-format csv -- python3 bench.py --config C4 --budget 65536 --steps 3 --warmup 1 --no-cpu --no-resident --no-probes > $O/kt_c4.log 2>&1 || { tail -20 $O/kt_c4.log; exit 1; }
head -4 $O/kt_c4/kt4_kernel_stats.csv
echo ALL_OK
