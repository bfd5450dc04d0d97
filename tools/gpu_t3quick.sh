# T3 change check: HBM-tier parity tests, then C4 at two budgets (product library)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1 || { echo TESTS_FAILED; tail -20 gpurun_out/t.log; exit 1; }
tail -1 gpurun_out/t.log
for b in 65536 1048576; do
  timeout -k 10 200 python -u tools/t3_prof.py $b > gpurun_out/q_$b.log 2>&1 || { echo "FAIL $b"; tail -5 gpurun_out/q_$b.log; exit 1; }
  echo "budget=$b $(tail -1 gpurun_out/q_$b.log)"
done
