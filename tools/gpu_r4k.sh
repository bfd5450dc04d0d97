# Round 4: k_spec validating its staged keys in-block -- the GPU suite, then
# the C2 bench line, kernel trace and FETCH_SIZE / WRITE_SIZE of k_spec.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r4k
mkdir -p $O/prof
step() { echo "== $1 $(date +%T)"; }
step tests
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|^E " $O/tests.log | head -20; exit 1; }
tail -1 $O/tests.log
PROF="--no-cpu --no-resident --no-probes --no-c3"
step bench_c2
timeout -k 10 300 python -u bench.py --steps 50 --warmup 5 $PROF > $O/bench_c2.json 2> $O/bench_c2.err || { tail -5 $O/bench_c2.err; exit 1; }
cut -c1-200 $O/bench_c2.json
step prof_c2
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof/kt_c2 -o kt --output-format csv -- python3 bench.py --steps 50 --warmup 5 $PROF > $O/prof/kt_c2.log 2>&1 || { tail -5 $O/prof/kt_c2.log; exit 1; }
step pmc_c2
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $O/prof/f_c2 -o f --output-format csv -- python3 bench.py --steps 5 --warmup 1 $PROF > $O/prof/f_c2.log 2>&1 || { tail -5 $O/prof/f_c2.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $O/prof/w_c2 -o w --output-format csv -- python3 bench.py --steps 5 --warmup 1 $PROF > $O/prof/w_c2.log 2>&1 || { tail -5 $O/prof/w_c2.log; exit 1; }
echo ALL_OK
