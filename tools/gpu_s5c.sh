# Records written at finish_key + fewer timing events: GPU suite, C2 bench;
# T3L pairs-in-flight A/B on C4 (UP = 2 default, 3, 4 variants).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/s5c
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|^E " $O/tests.log | head -30; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
timeout -k 10 200 python -u bench.py --steps 40 --warmup 5 --no-cpu --no-probes > $O/c2_$i.json 2> $O/c2_$i.err || { tail -5 $O/c2_$i.err; exit 1; }
python -c "import json;d=json.loads(open('$O/c2_$i.json').read().splitlines()[-1]);print('C2', round(d['value']/1e9,3),'Gops/s', round(d['ms_per_step'],4),'ms T0', round(d['tier0_ms'],4), 'res', round(d['resident']['ms_per_step'],4), d['resident']['same_records_as_d1'])"
done
for v in "" _up3 _up4 ""; do
  LINCHECK_LIB_OVERRIDE=$PWD/jepsen-etcd-demo_amd/lincheck/liblincheck$v.so timeout -k 10 300 python -u bench.py --config C4 --budget 65536 --steps 3 --warmup 1 --no-cpu --no-probes --no-resident > $O/c4$v.json 2> $O/c4$v.err || { tail -5 $O/c4$v.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/c4$v.json').read().splitlines()[-1]);print('C4 lib$v', round(d['ms_per_step'],3),'ms T3', round(d['tier3_ms'],3), d['verdicts'])"
done
echo ALL_OK
