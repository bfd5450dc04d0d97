# Round 6: lc_report's one-pass slot scan -- the counterexample parity tests
# (C5 at full size against the restatements) and the drop-in call's line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6z2; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_multi_register.py tests/test_gpu_parity.py  -v --timeout 300 --timeout-method thread > $O/parity.log 2>&1 || { grep -E "FAILED|Error" $O/parity.log | head; exit 1; }
tail -1 $O/parity.log
timeout -k 10 400 python -u bench.py --config C5 --jepsen --steps 10 --warmup 2 > $O/bench_c5_jepsen.json 2> $O/bench_c5_jepsen.err || { tail -5 $O/bench_c5_jepsen.err; exit 1; }
python -c "import json; d=json.loads(open('$O/bench_c5_jepsen.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['split_ms'], d['failures_equal_oracle'])"
