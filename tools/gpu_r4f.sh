# Round 4: the whole GPU suite, the C4 linear step (T3L), then the phase
# cycles (LC_WGL_PROF variant) on C2 / C4 and the C2 WGL bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=${OUT:-gpurun_out/r4f}
mkdir -p $O
echo "== tests $(date +%T)"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|^E " $O/tests.log | head -20; exit 1; }
tail -1 $O/tests.log
echo "== bench c4 linear $(date +%T)"
timeout -k 10 300 python -u bench.py --config C4 --budget 65536 --steps 3 --warmup 1 --no-resident --no-cpu > $O/bench_c4.json 2> $O/bench_c4.err || { tail -5 $O/bench_c4.err; exit 1; }
cut -c1-200 $O/bench_c4.json
echo "== bench $(date +%T)"
timeout -k 10 300 python -u bench.py --config C2 --algorithm wgl --steps 5 --warmup 1 --no-resident --no-c3 --no-cpu > $O/bench_c2_wgl.json 2> $O/bench_c2_wgl.err || { tail -5 $O/bench_c2_wgl.err; exit 1; }
cut -c1-200 $O/bench_c2_wgl.json
export LINCHECK_LIB_OVERRIDE=jepsen-etcd-demo_amd/lincheck/liblincheck_wglprof.so
for c in C2 C4; do
  b=1048576; [ $c = C4 ] && b=65536
  echo "== prof $c $(date +%T)"
  timeout -k 10 300 python -u tools/wgl_prof.py $c $b > $O/wglprof_$c.json 2> $O/wglprof_$c.err || { tail -5 $O/wglprof_$c.err; exit 1; }
  cat $O/wglprof_$c.json
done
echo ALL_OK
