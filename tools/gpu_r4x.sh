# Round 4: the speculative-segment tests with the rerun-grid case.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r4x
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_spec.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|^E " $O/tests.log | head -20; exit 1; }
grep -E "rerun|passed" $O/tests.log | tail -3
echo ALL_OK
