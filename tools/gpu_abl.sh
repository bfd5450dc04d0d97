set -o pipefail
cd "$GRAFT_REPO_ROOT"
for v in "" jepsen-etcd-demo_amd/lincheck/liblincheck_abl_GS.so; do
  echo "lib=$v"; LINCHECK_LIB_OVERRIDE=$v timeout -k 5 90 python tools/t0_run.py 0 300 || exit 1
  LINCHECK_LIB_OVERRIDE=$v timeout -k 5 90 python tools/t0_small.py 300 1000 10 | tail -1 || exit 1
done
