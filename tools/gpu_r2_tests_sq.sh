# Round 2, first GPU call: the whole -m gpu suite (new config / KAT tests
# included), then SQ counters of T0 on the bench's C2 step (verdicts-only
# FAST path), two passes of 8 SQ counters each.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/r2sq
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r2_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r2_tests.log; exit 1; }
tail -3 gpurun_out/r2_tests.log
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY -d gpurun_out/r2sq/p1 -o p1 -- python3 bench.py --no-cpu --steps 10 --warmup 2 > gpurun_out/r2sq/p1.log 2>&1 || { tail -20 gpurun_out/r2sq/p1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_BRANCH SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INSTS_VMEM SQ_ACTIVE_INST_LDS -d gpurun_out/r2sq/p2 -o p2 -- python3 bench.py --no-cpu --steps 10 --warmup 2 > gpurun_out/r2sq/p2.log 2>&1 || { tail -20 gpurun_out/r2sq/p2.log; exit 1; }
python3 tools/pmc_summary.py $(find gpurun_out/r2sq/p1 gpurun_out/r2sq/p2 -name "*.db" | sort) > gpurun_out/r2sq/summary.txt 2>&1 || true
cat gpurun_out/r2sq/summary.txt | cut -c1-400
