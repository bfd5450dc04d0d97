# Chunked lc_check_node: node tests, then the C3 20k shard D-1 with chunks
# (default) and without (LC_NODE_CHUNKS=1), and C2 (unchunked by size).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/chunks
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_node.py -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|^E " $O/tests.log | head -20; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u bench.py --config C3 --keys 20000 --steps 5 --warmup 1 --no-cpu > $O/c3s.json 2> $O/c3s.err || { tail -5 $O/c3s.err; exit 1; }
LC_NODE_CHUNKS=1 timeout -k 10 300 python -u bench.py --config C3 --keys 20000 --steps 5 --warmup 1 --no-cpu > $O/c3s_one.json 2> $O/c3s_one.err || { tail -5 $O/c3s_one.err; exit 1; }
timeout -k 10 300 python -u bench.py --config C3 --keys 12500 --steps 5 --warmup 1 --no-cpu > $O/c3_8th.json 2> $O/c3_8th.err || { tail -5 $O/c3_8th.err; exit 1; }
for f in c3s c3s_one c3_8th; do python -c "import json;d=json.load(open('$O/$f.json'));print('$f', round(d['ms_per_step'],3), '%.3g'%d['value'], 'resident', d['resident']['ms_per_step'], d['roofline']['avg_launch_ms'])"; done
echo ALL_OK
