set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
timeout -s KILL 90 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_IFETCH SQ_IFETCH_LEVEL SQ_INST_LEVEL_LDS SQ_WAIT_INST_LDS -d gpurun_out/pmc/p3 -o p3 -- python3 tools/t0_run.py 0 > gpurun_out/pmc/p3.log 2>&1 || { tail -20 gpurun_out/pmc/p3.log; exit 1; }
