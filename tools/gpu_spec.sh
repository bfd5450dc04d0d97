# Speculative segments: their GPU tests, the whole suite, C2 bench with and without.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/spec
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_spec.py -v -x --timeout 120 --timeout-method thread > $O/spec_tests.log 2>&1 || { echo SPEC_TESTS_FAILED; grep -E "FAILED|^E |Error" $O/spec_tests.log | head -30; tail -5 $O/spec_tests.log; exit 1; }
tail -1 $O/spec_tests.log
for s in 0 1; do
  LC_SPEC=$s timeout -k 10 300 python -u bench.py --steps 50 --warmup 5 --no-cpu > $O/bench_c2_spec$s.json 2> $O/bench_c2_spec$s.err || { tail -5 $O/bench_c2_spec$s.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_c2_spec$s.json'));print('spec=$s', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['resident']['ms_per_step'], d['parity_vs_oracle'])"
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|^E " $O/tests.log | head -30; exit 1; }
tail -1 $O/tests.log
