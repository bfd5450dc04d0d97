# Round 4: counter-free closure sweeps (T0) and WGL child adoption for narrow
# walks only -- the GPU suite, then the C2 default line, the C2 / C4 WGL lines,
# the C5 --jepsen line and the C2 WGL phase cycles.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r4p
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
step tests
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|^E " $O/tests.log | head -20; exit 1; }
tail -1 $O/tests.log
step bench_c2
timeout -k 10 400 python -u bench.py --steps 50 --warmup 5 > $O/bench_c2.json 2> $O/bench_c2.err || { tail -5 $O/bench_c2.err; exit 1; }
cut -c1-200 $O/bench_c2.json
step bench_c2_wgl
timeout -k 10 400 python -u bench.py --config C2 --algorithm wgl --steps 10 --warmup 2 --no-resident --no-c3 > $O/bench_c2_wgl.json 2> $O/bench_c2_wgl.err || { tail -5 $O/bench_c2_wgl.err; exit 1; }
step bench_c4_wgl
timeout -k 10 400 python -u bench.py --config C4 --budget 65536 --algorithm wgl --steps 3 --warmup 1 --no-resident > $O/bench_c4_wgl.json 2> $O/bench_c4_wgl.err || { tail -5 $O/bench_c4_wgl.err; exit 1; }
step bench_c5_jepsen
timeout -k 10 400 python -u bench.py --config C5 --jepsen --steps 10 --warmup 2 > $O/bench_c5_jepsen.json 2> $O/bench_c5_jepsen.err || { tail -5 $O/bench_c5_jepsen.err; exit 1; }
cut -c1-200 $O/bench_c5_jepsen.json
step wgl_phases
export LINCHECK_LIB_OVERRIDE=jepsen-etcd-demo_amd/lincheck/liblincheck_wglprof.so
timeout -k 10 300 python -u tools/wgl_prof.py C2 > $O/wglprof_C2.json 2> $O/wglprof_C2.err || { tail -5 $O/wglprof_C2.err; exit 1; }
cat $O/wglprof_C2.json
echo ALL_OK
