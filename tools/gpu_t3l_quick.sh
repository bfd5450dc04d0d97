# Layered HBM tier: its GPU tests, then per-key phase counts (variant) and
# C4 bench timing with it on and off.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/t3l
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_layers.py -x -v --timeout 200 --timeout-method thread > $O/tests_layers.log 2>&1 || { echo LAYER_TESTS_FAILED; grep -E "FAILED|^E |Error" $O/tests_layers.log | head -30; exit 1; }
tail -1 $O/tests_layers.log
LINCHECK_LIB_OVERRIDE=$PWD/jepsen-etcd-demo_amd/lincheck/liblincheck_t3lcnt.so timeout -k 10 200 python -u tools/t3l_cnt.py 65536 256 > $O/cnt.log 2>&1 || { tail -5 $O/cnt.log; exit 1; }
grep -v amdgpu.ids $O/cnt.log | cut -c1-400
timeout -k 10 300 python -u bench.py --config C4 --budget 65536 --steps 3 --warmup 1 --no-cpu > $O/bench_c4_layers.json 2> $O/bench_c4_layers.err || { tail -5 $O/bench_c4_layers.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench_c4_layers.json'));print('C4 2^16 step ms',d['ms_per_step'],'t3 ms',d['tier3_ms'])"
echo ALL_OK
