# A/B of whole bench steps (diagnostic): C2 bench line per lib variant
set -o pipefail
cd "$GRAFT_REPO_ROOT"
for v in "$@"; do
  LINCHECK_LIB_OVERRIDE=$v timeout -k 5 200 python bench.py --steps 200 --warmup 10 --no-cpu | python -c "import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print('lib=$v C2', '%.4g' % d['value'], 'step %.4f kernel %.4f t0 %.4f' % (d['ms_per_step'], d['kernel_ms'], d['tier0_ms']))" || exit 1
done
