# Speculative segments: tests, then a C2 sweep over segments per key and checkpoint distances.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/spec
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_spec.py -x -q --timeout 120 --timeout-method thread > $O/spec_tests.log 2>&1 || { echo SPEC_TESTS_FAILED; grep -E "FAILED|^E |Error" $O/spec_tests.log | head -30; tail -5 $O/spec_tests.log; exit 1; }
tail -1 $O/spec_tests.log
run() {  # label, env...
  local lab=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --steps 40 --warmup 5 --no-cpu --no-probes > $O/sw_$lab.json 2> $O/sw_$lab.err || { tail -5 $O/sw_$lab.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/sw_$lab.json'));print('$lab', round(d['value']/1e9,3), round(d['ms_per_step'],4), round(d['roofline']['avg_launch_ms'],4), round(d['resident']['ms_per_step'],4), d['parity_vs_oracle'])"
}
run plain LC_SPEC=0
run s4 LC_SPEC=1
run s2 LC_SPEC=1 LC_SPEC_SEGS=2
run s8 LC_SPEC=1 LC_SPEC_SEGS=8
run s4ck16 LC_SPEC=1 LC_SPEC_CK1=16 LC_SPEC_CK2=64
run s4ck48 LC_SPEC=1 LC_SPEC_CK1=48 LC_SPEC_CK2=200
