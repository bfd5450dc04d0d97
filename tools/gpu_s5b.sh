# events16 + reordered upload: GPU suite, C2 D-1 timing breakdown, C3-20k shard.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/s5b
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|^E " $O/tests.log | head -30; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
timeout -k 10 200 python -u bench.py --steps 40 --warmup 5 --no-cpu --no-probes > $O/c2_$i.json 2> $O/c2_$i.err || { tail -5 $O/c2_$i.err; exit 1; }
python -c "import json;d=json.loads(open('$O/c2_$i.json').read().splitlines()[-1]);print('C2', round(d['value']/1e9,3),'Gops/s', round(d['ms_per_step'],4),'ms T0', round(d['tier0_ms'],4), 'res', round(d['resident']['ms_per_step'],4), d['resident']['same_records_as_d1'])"
done
LC_TIMING=1 timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-cpu --no-probes --no-resident > $O/timing.json 2> $O/timing.err || exit 1
grep lc_check_node $O/timing.err | tail -3
timeout -k 10 300 python -u bench.py --config C3 --keys 20000 --steps 5 --warmup 1 --no-cpu --no-probes > $O/c3.json 2> $O/c3.err || { tail -5 $O/c3.err; exit 1; }
python -c "import json;d=json.loads(open('$O/c3.json').read().splitlines()[-1]);print('C3-20k', round(d['value']/1e9,3),'Gops/s', round(d['ms_per_step'],3),'ms T0', round(d['tier0_ms'],3), 'res', round(d['resident']['ms_per_step'],3))"
echo ALL_OK
