# Round 4: the T3L S' table at 1.5x its bound (LC_T3L_TSB 2) as the default --
# the GPU suite (test_gpu_layers: records identical with the layered tier on
# and off), then the C4 line and its kernel stats.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r4zd
mkdir -p $O/prof
echo "== tests $(date +%T)"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|^E " $O/tests.log | head -20; exit 1; }
tail -1 $O/tests.log
echo "== bench_c4 $(date +%T)"
timeout -k 10 300 python -u bench.py --config C4 --budget 65536 --steps 3 --warmup 1 > $O/bench_c4.json 2> $O/bench_c4.err || { tail -5 $O/bench_c4.err; exit 1; }
cut -c1-200 $O/bench_c4.json
echo "== prof_c4 $(date +%T)"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof/kt_c4 -o kt --output-format csv -- python3 bench.py --config C4 --budget 65536 --steps 3 --warmup 1 --no-cpu --no-resident --no-probes --no-c3 > $O/prof/kt_c4.log 2>&1 || { tail -20 $O/prof/kt_c4.log; exit 1; }
echo ALL_OK
