# Device validation of every batch: GPU suite, C4 step breakdown, C2 bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/s5e
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|^E " $O/tests.log | head -30; exit 1; }
tail -1 $O/tests.log
LC_TIMING=1 timeout -k 10 300 python -u bench.py --config C4 --budget 65536 --steps 3 --warmup 1 --no-cpu --no-probes --no-resident > $O/c4t.json 2> $O/c4t.err || { tail -5 $O/c4t.err; exit 1; }
grep lc_check_node $O/c4t.err | tail -3
python -c "import json;d=json.loads(open('$O/c4t.json').read().splitlines()[-1]);print('C4', round(d['ms_per_step'],3),'ms T3', round(d['tier3_ms'],3), d['verdicts'])"
timeout -k 10 200 python -u bench.py --steps 40 --warmup 5 --no-cpu --no-probes > $O/c2.json 2> $O/c2.err || { tail -5 $O/c2.err; exit 1; }
python -c "import json;d=json.loads(open('$O/c2.json').read().splitlines()[-1]);print('C2', round(d['value']/1e9,3),'Gops/s', round(d['ms_per_step'],4),'ms T0', round(d['tier0_ms'],4), 'res', round(d['resident']['ms_per_step'],4), d['resident']['same_records_as_d1'])"
echo ALL_OK
