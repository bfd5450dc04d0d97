# Layered HBM tier evidence: the whole GPU suite, the C4 bench line, a
# kernel-trace profile of it, and FETCH_SIZE / WRITE_SIZE passes of T3L.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/t3e
mkdir -p $O/prof
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|^E " $O/tests.log | head -20; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u bench.py --config C4 --budget 65536 --steps 5 --warmup 1 > $O/bench_c4.json 2> $O/bench_c4.err || { tail -5 $O/bench_c4.err; exit 1; }
cut -c1-200 $O/bench_c4.json
PROF="--no-cpu --no-resident --no-probes"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof/kt_c4 -o kt4 --output-format csv -- python3 bench.py --config C4 --budget 65536 --steps 3 --warmup 1 $PROF > $O/prof/kt_c4.log 2>&1 || { tail -20 $O/prof/kt_c4.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/prof/f_c4 -o f --output-format csv -- python3 bench.py --config C4 --budget 65536 --steps 2 --warmup 1 $PROF > $O/prof/f_c4.log 2>&1 || { tail -5 $O/prof/f_c4.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/prof/w_c4 -o w --output-format csv -- python3 bench.py --config C4 --budget 65536 --steps 2 --warmup 1 $PROF > $O/prof/w_c4.log 2>&1 || { tail -5 $O/prof/w_c4.log; exit 1; }
timeout -k 10 300 python -u bench.py --config C4 --budget 1048576 --steps 2 --warmup 1 --no-cpu > $O/bench_c4_b20.json 2> $O/bench_c4_b20.err || { tail -5 $O/bench_c4_b20.err; exit 1; }
cut -c1-200 $O/bench_c4_b20.json
echo ALL_OK
