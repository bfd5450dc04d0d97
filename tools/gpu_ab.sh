# A/B timing of T0 builds on the C2 batch (diagnostic): lib variants as args
set -o pipefail
cd "$GRAFT_REPO_ROOT"
for v in "$@"; do
  echo "lib=$v"; LINCHECK_LIB_OVERRIDE=$v timeout -k 5 90 python tools/t0_run.py 0 200 || exit 1
done
