# A/B timing of T0 builds (diagnostic): C2 T0 time, then a C3-shaped 20k-key
# bench line, for every lib variant given as an argument ("" = liblincheck.so)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
for v in "$@"; do
  echo "lib=$v"; LINCHECK_LIB_OVERRIDE=$v timeout -k 5 90 python tools/t0_run.py 0 200 || exit 1
  LINCHECK_LIB_OVERRIDE=$v timeout -k 5 200 python bench.py --config C3 --keys 20000 --steps 5 --warmup 1 --no-cpu | python -c "import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print('C3-20k', '%.3g' % d['value'], d['ms_per_step'])" || exit 1
done
