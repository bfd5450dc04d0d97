# Round-2 evidence: GPU suite, bench lines (C2 default, C5, C4, C3 shard, C1),
# rocprofv3 kernel-trace stats of the C2 and C4 bench commands (D-1 steps
# only, so every search launch in the trace is a timed-step launch),
# FETCH_SIZE / WRITE_SIZE passes, and a 2-rank rehearsal of the N > 1 path.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r2j
mkdir -p $O/prof
step() { echo "== $1"; }
step tests
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|^E " $O/tests.log | head -20; exit 1; }
tail -1 $O/tests.log
step bench_c2
timeout -k 10 300 python -u bench.py --steps 50 --warmup 5 > $O/bench_c2.json 2> $O/bench_c2.err || { tail -5 $O/bench_c2.err; exit 1; }
cut -c1-400 $O/bench_c2.json
step prof_c2
PROF="--no-cpu --no-resident --no-probes"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof/kt_c2 -o kt --output-format csv -- python3 bench.py --steps 50 --warmup 5 $PROF > $O/prof/kt_c2.log 2>&1 || { tail -20 $O/prof/kt_c2.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/prof/f_c2 -o f --output-format csv -- python3 bench.py --steps 5 --warmup 1 $PROF > $O/prof/f_c2.log 2>&1 || { tail -5 $O/prof/f_c2.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/prof/w_c2 -o w --output-format csv -- python3 bench.py --steps 5 --warmup 1 $PROF > $O/prof/w_c2.log 2>&1 || { tail -5 $O/prof/w_c2.log; exit 1; }
step bench_c5
timeout -k 10 300 python -u bench.py --config C5 --steps 20 --warmup 3 > $O/bench_c5.json 2> $O/bench_c5.err || { tail -5 $O/bench_c5.err; exit 1; }
step bench_c4
timeout -k 10 300 python -u bench.py --config C4 --budget 65536 --steps 3 --warmup 1 > $O/bench_c4.json 2> $O/bench_c4.err || { tail -5 $O/bench_c4.err; exit 1; }
step prof_c4
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof/kt_c4 -o kt4 --output-format csv -- python3 bench.py --config C4 --budget 65536 --steps 3 --warmup 1 $PROF > $O/prof/kt_c4.log 2>&1 || { tail -20 $O/prof/kt_c4.log; exit 1; }
step bench_c3_20k
timeout -k 10 300 python -u bench.py --config C3 --keys 20000 --steps 5 --warmup 1 --no-cpu > $O/bench_c3s.json 2> $O/bench_c3s.err || { tail -5 $O/bench_c3s.err; exit 1; }
step bench_c1
timeout -k 10 300 python -u bench.py --config C1 --steps 20 --warmup 3 > $O/bench_c1.json 2> $O/bench_c1.err || { tail -5 $O/bench_c1.err; exit 1; }
step rehearsal_n2
LC_BENCH_DEVICE=0 LC_BENCH_GATHER=host timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --keys 20000 --steps 5 --warmup 1 > $O/bench_n2_rehearsal.json 2> $O/bench_n2_rehearsal.err || { tail -20 $O/bench_n2_rehearsal.err; exit 1; }
cut -c1-300 $O/bench_n2_rehearsal.json
echo ALL_OK
