# Sanity pass on the current tree: the -m gpu suite, an optional register-tier
# A/B (SETTINGS), then the default bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/sanity
mkdir -p $O
if [ -n "$SETTINGS" ]; then
echo "== ab $(date +%T)"
timeout -k 10 300 python -u tools/spec_ab.py C2 1000 1000 $SETTINGS > $O/ab_c2.txt 2>&1 || { tail -5 $O/ab_c2.txt; exit 1; }
cat $O/ab_c2.txt
timeout -k 10 300 python -u tools/spec_ab.py C5 1000 1000 $SETTINGS > $O/ab_c5.txt 2>&1 || { tail -5 $O/ab_c5.txt; exit 1; }
cat $O/ab_c5.txt
fi
if [ -z "$NOTEST" ]; then
echo "== tests $(date +%T)"
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|^E " $O/tests.log | head -20; exit 1; }
tail -1 $O/tests.log
fi
if [ -z "$NOBENCH" ]; then
echo "== bench $(date +%T)"
timeout -k 10 400 python -u bench.py --steps 50 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
cut -c1-400 $O/bench.json
fi
echo ALL_OK
