# Round 4, first pass: the whole GPU suite, then bench lines of the new WGL
# path (C4 and C2 with --algorithm wgl, C4 competition), the drop-in's call
# (--jepsen, C5), and the FETCH_SIZE calibration (tools/fetch_calib.hip).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r4a
mkdir -p $O/prof
step() { echo "== $1 $(date +%T)"; }
if [ -z "$SKIP_TESTS" ]; then
step tests
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|^E " $O/tests.log | head -20; exit 1; }
tail -1 $O/tests.log
fi
step calib
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE -d $O/prof/calib -o calib --output-format csv -- ./tools/fetch_calib > $O/prof/calib.log 2>&1 || { tail -5 $O/prof/calib.log; exit 1; }
step bench_c4_wgl
timeout -k 10 400 python -u bench.py --config C4 --budget 65536 --algorithm wgl --steps 5 --warmup 1 --no-resident > $O/bench_c4_wgl.json 2> $O/bench_c4_wgl.err || { tail -5 $O/bench_c4_wgl.err; exit 1; }
cut -c1-400 $O/bench_c4_wgl.json
step bench_c2_wgl
timeout -k 10 400 python -u bench.py --config C2 --algorithm wgl --steps 10 --warmup 2 --no-resident > $O/bench_c2_wgl.json 2> $O/bench_c2_wgl.err || { tail -5 $O/bench_c2_wgl.err; exit 1; }
cut -c1-400 $O/bench_c2_wgl.json
step bench_c4_comp
timeout -k 10 400 python -u bench.py --config C4 --budget 65536 --algorithm competition --steps 3 --warmup 1 --no-resident --no-cpu > $O/bench_c4_comp.json 2> $O/bench_c4_comp.err || { tail -5 $O/bench_c4_comp.err; exit 1; }
step bench_c5_jepsen
timeout -k 10 400 python -u bench.py --config C5 --jepsen --steps 10 --warmup 2 > $O/bench_c5_jepsen.json 2> $O/bench_c5_jepsen.err || { tail -5 $O/bench_c5_jepsen.err; exit 1; }
cut -c1-600 $O/bench_c5_jepsen.json
echo ALL_OK
