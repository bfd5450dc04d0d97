# Pipelined D-1 (lc_check_node_async): node GPU tests, then the C2 / C5 / C4
# bench lines with the pipelined timed steps and the synchronous rate beside.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/pipe
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_node.py tests/test_gpu_configs.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|Error|^E " $O/tests.log | head -30; exit 1; }
tail -1 $O/tests.log
for c in C2 C5; do
  timeout -k 10 300 python -u bench.py --config $c --steps 50 --warmup 5 --no-cpu > $O/bench_$c.json 2> $O/bench_$c.err || { tail -5 $O/bench_$c.err; exit 1; }
  python -c "import json;d=json.load(open('$O/bench_$c.json'));print('$c', d['value'], d['ms_per_step'], d['d1_sync'], d['roofline']['avg_launch_ms'])"
done
timeout -k 10 300 python -u bench.py --config C4 --budget 65536 --steps 3 --warmup 1 --no-cpu > $O/bench_C4.json 2> $O/bench_C4.err || { tail -5 $O/bench_C4.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench_C4.json'));print('C4', d['value'], d['ms_per_step'], d['d1_sync'], d['roofline']['avg_launch_ms'])"
echo ALL_OK
