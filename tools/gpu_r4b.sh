# Round 4, WGL v2 pass: the WGL device tests on v2 (LDS cache tier, LDS frame
# ring, deferred inserts), then bench lines of the WGL step for v2 and for v1
# (the first device walk, built from the committed source as
# lincheck/liblincheck_wglv1.so, loaded through LINCHECK_LIB_OVERRIDE: A/B
# only), competition on C4, the drop-in's call on C5, FETCH_SIZE calibration.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r4b
mkdir -p $O/prof
step() { echo "== $1 $(date +%T)"; }
step tests
timeout -k 10 400 python -u -m pytest tests/test_gpu_wgl.py "tests/test_gpu_configs.py::test_wgl_on_device_against_wgl_restatement" "tests/test_gpu_configs.py::test_competition_on_device" -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|^E " $O/tests.log | head -20; exit 1; }
tail -1 $O/tests.log
step calib
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE -d $O/prof/calib -o calib --output-format csv -- ./tools/fetch_calib > $O/prof/calib.log 2>&1 || { tail -5 $O/prof/calib.log; exit 1; }
for v in v2 v1; do
  if [ $v = v1 ]; then export LINCHECK_LIB_OVERRIDE=jepsen-etcd-demo_amd/lincheck/liblincheck_wglv1.so; NC=--no-cpu; else unset LINCHECK_LIB_OVERRIDE; NC=; fi
  step bench_c2_wgl_$v
  timeout -k 10 400 python -u bench.py --config C2 --algorithm wgl --steps 5 --warmup 1 --no-resident --no-c3 $NC > $O/bench_c2_wgl_$v.json 2> $O/bench_c2_wgl_$v.err || { tail -5 $O/bench_c2_wgl_$v.err; exit 1; }
  cut -c1-300 $O/bench_c2_wgl_$v.json
  step bench_c4_wgl_$v
  timeout -k 10 400 python -u bench.py --config C4 --budget 65536 --algorithm wgl --steps 3 --warmup 1 --no-resident $NC > $O/bench_c4_wgl_$v.json 2> $O/bench_c4_wgl_$v.err || { tail -5 $O/bench_c4_wgl_$v.err; exit 1; }
  cut -c1-300 $O/bench_c4_wgl_$v.json
done
unset LINCHECK_LIB_OVERRIDE
step bench_c4_comp
timeout -k 10 400 python -u bench.py --config C4 --budget 65536 --algorithm competition --steps 3 --warmup 1 --no-resident --no-cpu > $O/bench_c4_comp.json 2> $O/bench_c4_comp.err || { tail -5 $O/bench_c4_comp.err; exit 1; }
step bench_c5_jepsen
timeout -k 10 400 python -u bench.py --config C5 --jepsen --steps 10 --warmup 2 > $O/bench_c5_jepsen.json 2> $O/bench_c5_jepsen.err || { tail -5 $O/bench_c5_jepsen.err; exit 1; }
cut -c1-600 $O/bench_c5_jepsen.json
echo ALL_OK
