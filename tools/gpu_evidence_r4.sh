# Round-4 evidence: GPU suite; bench lines (C2 default with c3_strong, C5, the
# C3 per-GPU shard, C4 at 2^16 linear / WGL / competition, C2 WGL, C5 --jepsen);
# rocprofv3 kernel stats of the C2, C3-shard, C4 and C4-WGL commands; FETCH_SIZE
# / WRITE_SIZE and SQ passes of C2's k_spec, the C3 shard's k_spec<2, 2> and C4's
# T3L (profiles/ JSONs tagged round 4, the only ones bench.py quotes).
# PART=A: tests, C2, C5, C3 shard; PART=B: C4 (linear / WGL / competition),
# C2 WGL, C5 --jepsen (each part within one gpurun call's limit).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r4
mkdir -p $O/prof
step() { echo "== $1 $(date +%T)"; }
if [ -z "$SKIP_TESTS" ]; then
step tests
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|^E " $O/tests.log | head -20; exit 1; }
tail -1 $O/tests.log
fi
if [ "${PART:-all}" != B ]; then
step bench_c2
timeout -k 10 400 python -u bench.py --steps 50 --warmup 5 > $O/bench_c2.json 2> $O/bench_c2.err || { tail -5 $O/bench_c2.err; exit 1; }
cut -c1-300 $O/bench_c2.json
fi
PROF="--no-cpu --no-resident --no-probes --no-c3"
SQ1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU"
SQ2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_SMEM"
prof() {  # name, bench args
  local n=$1; shift
  step prof_$n
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof/kt_$n -o kt --output-format csv -- python3 bench.py "$@" > $O/prof/kt_$n.log 2>&1 || { tail -20 $O/prof/kt_$n.log; return 1; }
}
pmc() {  # name, bench args (short runs)
  local n=$1; shift
  step pmc_$n
  timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $O/prof/f_$n -o f --output-format csv -- python3 bench.py "$@" > $O/prof/f_$n.log 2>&1 || { tail -5 $O/prof/f_$n.log; return 1; }
  timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $O/prof/w_$n -o w --output-format csv -- python3 bench.py "$@" > $O/prof/w_$n.log 2>&1 || { tail -5 $O/prof/w_$n.log; return 1; }
  timeout -s KILL 150 rocprofv3 --pmc $SQ1 -d $O/prof/sq1_$n -o p1 --output-format csv -- python3 bench.py "$@" > $O/prof/sq1_$n.log 2>&1 || { tail -5 $O/prof/sq1_$n.log; return 1; }
  timeout -s KILL 150 rocprofv3 --pmc $SQ2 -d $O/prof/sq2_$n -o p2 --output-format csv -- python3 bench.py "$@" > $O/prof/sq2_$n.log 2>&1 || { tail -5 $O/prof/sq2_$n.log; return 1; }
}
if [ "${PART:-all}" != B ]; then
prof c2 --steps 50 --warmup 5 $PROF || exit 1
pmc c2 --steps 5 --warmup 1 $PROF || exit 1
step bench_c5
timeout -k 10 300 python -u bench.py --config C5 --steps 20 --warmup 3 > $O/bench_c5.json 2> $O/bench_c5.err || { tail -5 $O/bench_c5.err; exit 1; }
step bench_c3_shard
timeout -k 10 300 python -u bench.py --config C3 --keys 12500 --steps 10 --warmup 2 --no-cpu > $O/bench_c3s.json 2> $O/bench_c3s.err || { tail -5 $O/bench_c3s.err; exit 1; }
prof c3s --config C3 --keys 12500 --steps 10 --warmup 2 $PROF || exit 1
pmc c3s --config C3 --keys 12500 --steps 3 --warmup 1 $PROF || exit 1
fi
if [ "${PART:-all}" != A ]; then
step bench_c4
timeout -k 10 300 python -u bench.py --config C4 --budget 65536 --steps 3 --warmup 1 > $O/bench_c4.json 2> $O/bench_c4.err || { tail -5 $O/bench_c4.err; exit 1; }
prof c4 --config C4 --budget 65536 --steps 3 --warmup 1 $PROF || exit 1
pmc c4 --config C4 --budget 65536 --steps 2 --warmup 1 $PROF || exit 1
step bench_c4_wgl
timeout -k 10 400 python -u bench.py --config C4 --budget 65536 --algorithm wgl --steps 3 --warmup 1 --no-resident > $O/bench_c4_wgl.json 2> $O/bench_c4_wgl.err || { tail -5 $O/bench_c4_wgl.err; exit 1; }
prof c4wgl --config C4 --budget 65536 --algorithm wgl --steps 3 --warmup 1 $PROF || exit 1
step bench_c4_comp
timeout -k 10 400 python -u bench.py --config C4 --budget 65536 --algorithm competition --steps 3 --warmup 1 --no-resident --no-cpu > $O/bench_c4_comp.json 2> $O/bench_c4_comp.err || { tail -5 $O/bench_c4_comp.err; exit 1; }
step bench_c2_wgl
timeout -k 10 400 python -u bench.py --config C2 --algorithm wgl --steps 10 --warmup 2 --no-resident --no-c3 > $O/bench_c2_wgl.json 2> $O/bench_c2_wgl.err || { tail -5 $O/bench_c2_wgl.err; exit 1; }
prof c2wgl --config C2 --algorithm wgl --steps 10 --warmup 2 $PROF || exit 1
step bench_c5_jepsen
timeout -k 10 400 python -u bench.py --config C5 --jepsen --steps 10 --warmup 2 > $O/bench_c5_jepsen.json 2> $O/bench_c5_jepsen.err || { tail -5 $O/bench_c5_jepsen.err; exit 1; }
step wgl_phases
( export LINCHECK_LIB_OVERRIDE=jepsen-etcd-demo_amd/lincheck/liblincheck_wglprof.so
  timeout -k 10 300 python -u tools/wgl_prof.py C2 > $O/wglprof_C2.json 2> $O/wglprof_C2.err &&
  timeout -k 10 300 python -u tools/wgl_prof.py C4 65536 > $O/wglprof_C4.json 2> $O/wglprof_C4.err ) || { tail -5 $O/wglprof_C2.err $O/wglprof_C4.err; exit 1; }
fi
echo ALL_OK
