# Round 4, WGL v3 pass: the whole GPU suite on the build (k_spec LDS staging,
# WGL v3), then the WGL step on C2 and C4, an A/B of k_spec's LDS staging
# (LC_PATH_SPEC_NOSTAGE) on C2, the drop-in's call on C5, and a kernel trace
# of the C2 WGL step.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r4c
mkdir -p $O/prof
step() { echo "== $1 $(date +%T)"; }
step tests
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|^E " $O/tests.log | head -20; exit 1; }
tail -1 $O/tests.log
step bench_c2_wgl
timeout -k 10 400 python -u bench.py --config C2 --algorithm wgl --steps 5 --warmup 1 --no-resident --no-c3 --no-cpu > $O/bench_c2_wgl.json 2> $O/bench_c2_wgl.err || { tail -5 $O/bench_c2_wgl.err; exit 1; }
cut -c1-300 $O/bench_c2_wgl.json
step bench_c4_wgl
timeout -k 10 400 python -u bench.py --config C4 --budget 65536 --algorithm wgl --steps 3 --warmup 1 --no-resident --no-cpu > $O/bench_c4_wgl.json 2> $O/bench_c4_wgl.err || { tail -5 $O/bench_c4_wgl.err; exit 1; }
cut -c1-300 $O/bench_c4_wgl.json
for f in 0 0x1000; do
  step bench_c2_spec_$f
  timeout -k 10 400 python -u bench.py --config C2 --steps 20 --warmup 3 --no-resident --no-c3 --no-cpu --no-probes --path-flags $f > $O/bench_c2_spec_$f.json 2> $O/bench_c2_spec_$f.err || { tail -5 $O/bench_c2_spec_$f.err; exit 1; }
  cut -c1-300 $O/bench_c2_spec_$f.json
done
step bench_c5_jepsen
timeout -k 10 400 python -u bench.py --config C5 --jepsen --steps 10 --warmup 2 --no-cpu > $O/bench_c5_jepsen.json 2> $O/bench_c5_jepsen.err || { tail -5 $O/bench_c5_jepsen.err; exit 1; }
cut -c1-600 $O/bench_c5_jepsen.json
step prof_c2_wgl
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof/c2wgl -o c2wgl --output-format csv -- python3 bench.py --config C2 --algorithm wgl --steps 3 --warmup 1 --no-resident --no-c3 --no-cpu > $O/prof/c2wgl.log 2>&1 || { tail -5 $O/prof/c2wgl.log; exit 1; }
echo ALL_OK
