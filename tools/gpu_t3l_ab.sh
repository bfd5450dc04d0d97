# T3L fused-step sizing A/B on C4 (budget 2^16): EST 3 (default), 2, 1.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/t3lab
mkdir -p $O
for rep in 1 2 3; do
for v in "" _e2 _e1; do
  LINCHECK_LIB_OVERRIDE=$PWD/jepsen-etcd-demo_amd/lincheck/liblincheck$v.so timeout -k 10 300 python -u bench.py --config C4 --budget 65536 --steps 3 --warmup 1 --no-cpu --no-probes --no-resident > $O/c4$v.json 2> $O/c4$v.err || { tail -5 $O/c4$v.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/c4$v.json').read().splitlines()[-1]);print('C4 lib$v', round(d['ms_per_step'],3),'ms T3', round(d['tier3_ms'],3), d['verdicts'])"
done
done
LINCHECK_LIB_OVERRIDE=$PWD/jepsen-etcd-demo_amd/lincheck/liblincheck_e1.so timeout -k 10 300 python -u -m pytest tests/test_gpu_layers.py tests/test_gpu_configs.py -q -x -k "layers or c4" --timeout 200 --timeout-method thread > $O/t.log 2>&1 || { tail -20 $O/t.log; exit 1; }
tail -1 $O/t.log
echo ALL_OK
