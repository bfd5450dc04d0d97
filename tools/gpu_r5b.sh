set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r5d
mkdir -p $O
echo "== pack $(date +%T)"
LC_TIMING=1 timeout -k 10 300 python -u tools/pack_timing.py > $O/pack.json 2> $O/pack.err || { tail -5 $O/pack.err; exit 1; }
tail -1 $O/pack.json | cut -c1-1800
echo "== probe $(date +%T)"
timeout -k 10 120 ./tools/probe/pin_probe 660 > $O/pin.json 2>&1 || { cat $O/pin.json; exit 1; }
cat $O/pin.json
echo "== jprof $(date +%T)"
timeout -k 10 200 python -u tools/jepsen_profile.py > $O/jprof.txt 2>&1 || { tail -5 $O/jprof.txt; exit 1; }
head -60 $O/jprof.txt
echo "== tests $(date +%T)"
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|^E " $O/tests.log | head -20; exit 1; }
tail -1 $O/tests.log
echo "== jepsen $(date +%T)"
timeout -k 10 300 python -u bench.py --config C5 --jepsen --steps 10 --warmup 2 > $O/jepsen.json 2> $O/jepsen.err || { tail -5 $O/jepsen.err; exit 1; }
cut -c1-1200 $O/jepsen.json
echo "== bench $(date +%T)"
timeout -k 10 400 python -u bench.py --steps 50 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['pack_ms'], d['c3_strong'] and {k: d['c3_strong'][k] for k in ('pack_ms','ms_per_step','ops_per_s')})"
echo ALL_OK
