# C4 evidence after T3L changes: GPU suite, bench C4 at 2^16 and 2^20,
# rocprofv3 kernel stats of the C4 command.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r3c
mkdir -p $O/prof
echo "== tests $(date +%T)"
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|^E " $O/tests.log | head -20; exit 1; }
tail -1 $O/tests.log
PROF="--no-cpu --no-resident --no-probes --no-c3"
echo "== bench_c4 $(date +%T)"
timeout -k 10 300 python -u bench.py --config C4 --budget 65536 --steps 3 --warmup 1 > $O/bench_c4.json 2> $O/bench_c4.err || { tail -5 $O/bench_c4.err; exit 1; }
echo "== prof_c4 $(date +%T)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof/kt_c4 -o kt4 --output-format csv -- python3 bench.py --config C4 --budget 65536 --steps 3 --warmup 1 $PROF > $O/prof/kt_c4.log 2>&1 || { tail -20 $O/prof/kt_c4.log; exit 1; }
echo "== bench_c4_b20 $(date +%T)"
timeout -k 10 400 python -u bench.py --config C4 --budget 1048576 --steps 2 --warmup 1 --no-resident > $O/bench_c4_b20.json 2> $O/bench_c4_b20.err || { tail -5 $O/bench_c4_b20.err; exit 1; }
echo ALL_OK
