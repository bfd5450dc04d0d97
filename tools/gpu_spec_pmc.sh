# SQ counters of the speculative-segment kernel on C2 (two passes).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/specpmc
mkdir -p $O
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM -d $O/p1 -o p1 -- python3 tools/spec_run.py 3 > $O/p1.log 2>&1 || { tail -20 $O/p1.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_BRANCH SQ_WAIT_ANY SQ_INSTS_LDS SQ_INST_CYCLES_SALU SQ_IFETCH SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC -d $O/p2 -o p2 -- python3 tools/spec_run.py 3 > $O/p2.log 2>&1 || { tail -20 $O/p2.log; exit 1; }
python3 tools/pmc_summary.py $(find $O/p1 $O/p2 -name "*.db" | sort) | grep -i "k_spec"
