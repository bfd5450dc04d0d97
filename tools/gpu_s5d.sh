# GPU suite after the kernel cleanup + the C4 D-1 step breakdown.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/s5d
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|^E " $O/tests.log | head -30; exit 1; }
tail -1 $O/tests.log
LC_TIMING=1 timeout -k 10 300 python -u bench.py --config C4 --budget 65536 --steps 3 --warmup 1 --no-cpu --no-probes --no-resident > $O/c4t.json 2> $O/c4t.err || { tail -5 $O/c4t.err; exit 1; }
grep lc_check_node $O/c4t.err | tail -3
python -c "import json;d=json.loads(open('$O/c4t.json').read().splitlines()[-1]);print('C4', round(d['ms_per_step'],3),'ms T3', round(d['tier3_ms'],3), 'T0', d['tier0_ms'])"
echo ALL_OK
