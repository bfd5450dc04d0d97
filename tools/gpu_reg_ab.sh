# A/B of the 9-10-pending closure in VGPRs (default: both), 9 only (r8), neither (r0).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/regab
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_spec.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS_FAILED; tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2; do
for v in "" _r8 _r0; do
  LINCHECK_LIB_OVERRIDE=$PWD/jepsen-etcd-demo_amd/lincheck/liblincheck$v.so timeout -k 10 200 python -u bench.py --steps 40 --warmup 5 --no-cpu --no-probes > $O/c2$v.json 2> $O/c2$v.err || { tail -5 $O/c2$v.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/c2$v.json').read().splitlines()[-1]);print('C2 lib$v', round(d['value']/1e9,3),'Gops/s', round(d['ms_per_step'],4),'ms T0', round(d['tier0_ms'],4), 'res', round(d['resident']['ms_per_step'],4), d['parity_vs_oracle'], d['resident']['same_records_as_d1'])"
done
done
echo ALL_OK
