# The -m gpu suite (one pytest process), each test bounded; log under gpurun_out/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread ${1:-} > gpurun_out/tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR" gpurun_out/tests.log | grep -v PASSED | head -30
tail -3 gpurun_out/tests.log
exit $rc
