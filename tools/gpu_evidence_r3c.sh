# Round-3 evidence, final pass (exact-set segments, rerun launch): GPU suite,
# bench lines (C2 default with c3_strong, C5, C3 per-GPU shard), rocprofv3
# kernel stats of the C2 command (D-1 steps only), FETCH_SIZE / WRITE_SIZE and
# SQ passes of the C2 search kernel -> profiles/ JSONs the bench reads.
# (C4, C1 and the N = 2 rehearsal: gpu_evidence_c4.sh / gpu_evidence_r3b.sh.)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r3c
mkdir -p $O/prof
step() { echo "== $1 $(date +%T)"; }
if [ -z "$SKIP_TESTS" ]; then
step tests
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|^E " $O/tests.log | head -20; exit 1; }
tail -1 $O/tests.log
fi
step bench_c2
timeout -k 10 400 python -u bench.py --steps 50 --warmup 5 > $O/bench_c2.json 2> $O/bench_c2.err || { tail -5 $O/bench_c2.err; exit 1; }
cut -c1-300 $O/bench_c2.json
PROF="--no-cpu --no-resident --no-probes --no-c3"
step prof_c2
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof/kt_c2 -o kt --output-format csv -- python3 bench.py --steps 50 --warmup 5 $PROF > $O/prof/kt_c2.log 2>&1 || { tail -20 $O/prof/kt_c2.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/prof/f_c2 -o f --output-format csv -- python3 bench.py --steps 5 --warmup 1 $PROF > $O/prof/f_c2.log 2>&1 || { tail -5 $O/prof/f_c2.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/prof/w_c2 -o w --output-format csv -- python3 bench.py --steps 5 --warmup 1 $PROF > $O/prof/w_c2.log 2>&1 || { tail -5 $O/prof/w_c2.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU -d $O/prof/sq1_c2 -o p1 --output-format csv -- python3 bench.py --steps 5 --warmup 1 $PROF > $O/prof/sq1_c2.log 2>&1 || { tail -5 $O/prof/sq1_c2.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_SMEM -d $O/prof/sq2_c2 -o p2 --output-format csv -- python3 bench.py --steps 5 --warmup 1 $PROF > $O/prof/sq2_c2.log 2>&1 || { tail -5 $O/prof/sq2_c2.log; exit 1; }
step bench_c5
timeout -k 10 300 python -u bench.py --config C5 --steps 20 --warmup 3 > $O/bench_c5.json 2> $O/bench_c5.err || { tail -5 $O/bench_c5.err; exit 1; }
step bench_c3_shard
timeout -k 10 300 python -u bench.py --config C3 --keys 12500 --steps 10 --warmup 2 --no-cpu > $O/bench_c3s.json 2> $O/bench_c3s.err || { tail -5 $O/bench_c3s.err; exit 1; }
echo ALL_OK
