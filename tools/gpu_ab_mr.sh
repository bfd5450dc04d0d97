# A/B: product library vs a variant on the C2 bench (T0), with the variant's parity tests first
set -o pipefail
cd "$GRAFT_REPO_ROOT"
V=$GRAFT_REPO_ROOT/jepsen-etcd-demo_amd/lincheck/liblincheck_${1}.so
LINCHECK_LIB_OVERRIDE=$V timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "c2 or c5 or fast or resident or small or budget or counterexamples" > gpurun_out/ab_t.log 2>&1 || { echo VARIANT_TESTS_FAILED; tail -20 gpurun_out/ab_t.log; exit 1; }
tail -1 gpurun_out/ab_t.log
for r in 1 2; do
for v in "" $V; do
  LINCHECK_LIB_OVERRIDE=$v timeout -k 5 200 python bench.py --steps 200 --warmup 10 --no-cpu | python -c "import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print('lib=${v##*/}', '%.4g' % d['value'], 'step %.4f kernel %.4f t0 %.4f' % (d['ms_per_step'], d['kernel_ms'], d['tier0_ms']))" || exit 1
done
done
