# Pipelined step with records written straight into mapped host memory:
# node tests, smoke, C2 A/B (direct vs staged download), C5.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/direct
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_node.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|Error|^E " $O/tests.log | head -30; exit 1; }
tail -1 $O/tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for v in direct staged direct; do
  if [ $v = staged ]; then export LC_NODE_STAGED=1; else unset LC_NODE_STAGED; fi
  timeout -k 10 300 python -u bench.py --steps 200 --warmup 10 --no-cpu --no-resident --no-probes > $O/bench_$v.json 2> $O/bench_$v.err || { tail -5 $O/bench_$v.err; exit 1; }
  python -c "import json;d=json.load(open('$O/bench_$v.json'));print('$v', d['value'], d['ms_per_step'], d['d1_sync']['ms_per_step'], d['d1_sync']['same_records'])"
done
echo ALL_OK
