# SQ counters of T0 on the C2 batch (diagnostic), two passes; arg: lib variant
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
L=${1:-}
LINCHECK_LIB_OVERRIDE=$L timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM -d gpurun_out/pmc/p1 -o p1 -- python3 tools/t0_run.py 0 4 > gpurun_out/pmc/p1.log 2>&1 || { tail -20 gpurun_out/pmc/p1.log; exit 1; }
LINCHECK_LIB_OVERRIDE=$L timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_BRANCH SQ_WAIT_ANY SQ_INSTS_LDS SQ_INST_CYCLES_SALU SQ_IFETCH SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC -d gpurun_out/pmc/p2 -o p2 -- python3 tools/t0_run.py 0 4 > gpurun_out/pmc/p2.log 2>&1 || { tail -20 gpurun_out/pmc/p2.log; exit 1; }
python3 tools/pmc_summary.py $(find gpurun_out/pmc/p1 gpurun_out/pmc/p2 -name "*.db" | sort) | grep -i lattice
