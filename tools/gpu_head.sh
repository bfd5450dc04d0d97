# Quick state check: GPU suite + C2 bench on the current tree.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/head
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|^E " $O/tests.log | head -30; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u bench.py --steps 50 --warmup 5 > $O/bench_c2.json 2> $O/bench_c2.err || { tail -5 $O/bench_c2.err; exit 1; }
cut -c1-600 $O/bench_c2.json
