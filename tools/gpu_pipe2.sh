# Pipelined D-1 on large shards (no chunking, whole upload overlapping the
# previous search): node tests, C3 shard bench, 2-rank rehearsal.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/pipe2
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_node.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|Error|^E " $O/tests.log | head -30; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u bench.py --config C3 --keys 20000 --steps 5 --warmup 1 --no-cpu > $O/bench_c3s.json 2> $O/bench_c3s.err || { tail -5 $O/bench_c3s.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench_c3s.json'));print('C3s', d['value'], d['ms_per_step'], d['d1_sync'], d['roofline']['avg_launch_ms'], d['resident'])"
LC_BENCH_DEVICE=0 LC_BENCH_GATHER=host timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --keys 20000 --steps 5 --warmup 1 > $O/bench_n2.json 2> $O/bench_n2.err || { tail -20 $O/bench_n2.err; exit 1; }
grep metric $O/bench_n2.json | python -c "import json,sys;d=json.loads(sys.stdin.read());print('N2', d['value'], d['ms_per_step'], d['d1_sync'])"
echo ALL_OK
