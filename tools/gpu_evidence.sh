# The round's GPU evidence, one parametrised script (replaces round 3-4's
# one-off gpu_r4*.sh / gpu_evidence_r*.sh): the GPU suite, bench lines,
# rocprofv3 kernel stats, and FETCH_SIZE / WRITE_SIZE and SQ passes of each
# line's dominant kernel.  tools/collect_evidence.sh then writes profiles/.
#
#   PARTS="tests c2 c5 c3s c4 c4wgl c2wgl c4comp c5jepsen" R=5 bash tools/gpu_evidence.sh
#
# Each part is one workload; every GPU step runs under its own time limit and
# the script stops at the first failure.  O=gpurun_out/r$R.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=${R:-5}
O=gpurun_out/r$R
mkdir -p $O/prof
PARTS=${PARTS:-"tests c2 c5 c3s c4 c4wgl c2wgl c4comp c5jepsen c4wgl24"}
step() { echo "== $1 $(date +%T)"; }
PROF="--no-cpu --no-resident --no-probes --no-c3"
SQ1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU"
SQ2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_SMEM"
bench() {  # name limit args...
  local n=$1 lim=$2; shift 2
  step bench_$n
  timeout -k 10 $lim python -u bench.py "$@" > $O/bench_$n.json 2> $O/bench_$n.err || { tail -5 $O/bench_$n.err; exit 1; }
  cut -c1-300 $O/bench_$n.json
}
prof() {  # name limit bench args: kernel trace + stats
  local n=$1 lim=$2; shift 2
  step prof_$n
  timeout -k 10 $lim rocprofv3 --kernel-trace --stats -d $O/prof/kt_$n -o kt --output-format csv -- python3 bench.py "$@" > $O/prof/kt_$n.log 2>&1 || { tail -20 $O/prof/kt_$n.log; exit 1; }
}
pmc() {  # name bench args: 4 counter passes, each its own run
  local n=$1; shift
  step pmc_$n
  timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d $O/prof/f_$n -o f --output-format csv -- python3 bench.py "$@" > $O/prof/f_$n.log 2>&1 || { tail -5 $O/prof/f_$n.log; exit 1; }
  timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d $O/prof/w_$n -o w --output-format csv -- python3 bench.py "$@" > $O/prof/w_$n.log 2>&1 || { tail -5 $O/prof/w_$n.log; exit 1; }
  timeout -s KILL 200 rocprofv3 --pmc $SQ1 -d $O/prof/sq1_$n -o p1 --output-format csv -- python3 bench.py "$@" > $O/prof/sq1_$n.log 2>&1 || { tail -5 $O/prof/sq1_$n.log; exit 1; }
  timeout -s KILL 200 rocprofv3 --pmc $SQ2 -d $O/prof/sq2_$n -o p2 --output-format csv -- python3 bench.py "$@" > $O/prof/sq2_$n.log 2>&1 || { tail -5 $O/prof/sq2_$n.log; exit 1; }
}
for part in $PARTS; do
  case $part in
  tests)
    step tests
    timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|^E " $O/tests.log | head -20; exit 1; }
    tail -1 $O/tests.log ;;
  c2)
    bench c2 400 --steps 50 --warmup 5
    prof c2 400 --steps 50 --warmup 5 $PROF
    pmc c2 --steps 5 --warmup 1 $PROF ;;
  c5)
    bench c5 300 --config C5 --steps 20 --warmup 3
    prof c5 300 --config C5 --steps 20 --warmup 3 $PROF ;;
  c3s)
    bench c3s 300 --config C3 --keys 12500 --steps 10 --warmup 2 --no-cpu
    prof c3s 300 --config C3 --keys 12500 --steps 10 --warmup 2 $PROF
    pmc c3s --config C3 --keys 12500 --steps 3 --warmup 1 $PROF ;;
  c4)
    bench c4 300 --config C4 --budget 65536 --steps 3 --warmup 1
    prof c4 300 --config C4 --budget 65536 --steps 3 --warmup 1 $PROF
    pmc c4 --config C4 --budget 65536 --steps 2 --warmup 1 $PROF ;;
  c4wgl)
    bench c4_wgl 400 --config C4 --budget 65536 --algorithm wgl --steps 3 --warmup 1 --no-resident
    prof c4wgl 400 --config C4 --budget 65536 --algorithm wgl --steps 3 --warmup 1 $PROF
    pmc c4wgl --config C4 --budget 65536 --algorithm wgl --steps 1 --warmup 1 $PROF ;;
  c2wgl)
    bench c2_wgl 400 --config C2 --algorithm wgl --steps 10 --warmup 2 --no-resident --no-c3
    prof c2wgl 400 --config C2 --algorithm wgl --steps 10 --warmup 2 $PROF
    pmc c2wgl --config C2 --algorithm wgl --steps 3 --warmup 1 $PROF ;;
  c4comp)
    bench c4_comp 400 --config C4 --budget 65536 --algorithm competition --steps 3 --warmup 1 --no-resident --no-cpu ;;
  c1)
    bench c1 200 --config C1 --steps 20 --warmup 3 ;;
  c5jepsen)
    bench c5_jepsen 400 --config C5 --jepsen --steps 10 --warmup 2 ;;
  c4wgl24)
    # BASELINE C4 decided: knossos.wgl's walk at a 2^24 cache budget
    # (profiles/r05_c4_budget_sweep.json: every key valid there)
    # (--cpu-full: oracle/wgl_ref.c on all 256 keys beside it)
    bench c4_wgl24 900 --config C4 --budget 16777216 --algorithm wgl --d1-sync --steps 1 --warmup 1 --no-resident --cpu-full ;;
  *) echo "unknown part $part"; exit 2 ;;
  esac
done
echo ALL_OK
