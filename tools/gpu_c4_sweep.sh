# the C4 budget sweep (tests/tools/c4_budget_sweep.py) -- :wgl and
# :linear on full C4 at 2^16 .. 2^22 with the C oracles on a 16-key sample,
# then :wgl at 2^24 (device only).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/c4sweep
mkdir -p $O
echo "== wgl $(date +%T)"
timeout -k 10 420 python -u tests/tools/c4_budget_sweep.py --algos wgl --budgets 16,18,20,22 --sample 16 --out $O/wgl.json > $O/wgl.log 2>&1 || { tail -5 $O/wgl.log; exit 1; }
tail -4 $O/wgl.log | cut -c1-400
echo "== linear $(date +%T)"
timeout -k 10 420 python -u tests/tools/c4_budget_sweep.py --algos linear --budgets 16,18,20,22 --sample 16 --out $O/linear.json > $O/linear.log 2>&1 || { tail -5 $O/linear.log; exit 1; }
tail -4 $O/linear.log | cut -c1-400
echo "== wgl24 $(date +%T)"
timeout -k 10 240 python -u tests/tools/c4_budget_sweep.py --algos wgl --budgets 24 --sample 0 --out $O/wgl24.json > $O/wgl24.log 2>&1 || { tail -5 $O/wgl24.log; exit 1; }
tail -2 $O/wgl24.log | cut -c1-400
echo ALL_OK
