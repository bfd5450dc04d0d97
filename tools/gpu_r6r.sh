# Round 6: 8 exact segments per key for small Jepsen-shaped batches -- the
# register-tier and parity GPU tests, and the C5 / C2 drop-in call lines.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6r; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_spec.py tests/test_gpu_segments.py tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -u bench.py --config C5 --jepsen --steps 10 --warmup 2 > $O/c5j.json 2> $O/c5j.err || { tail $O/c5j.err; exit 1; }
timeout -k 10 300 python -u bench.py --config C2 --jepsen --steps 10 --warmup 2 > $O/c2j.json 2> $O/c2j.err || { tail $O/c2j.err; exit 1; }
for f in c5j c2j; do python3 -c "import json; d=json.loads(open('$O/$f.json').read().strip().splitlines()[-1]); print('$f', round(d['ms_per_step'],3), d['split_ms'], d['search_stats'], d['failures_equal_oracle'])"; done
