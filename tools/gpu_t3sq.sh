# SQ counters of the HBM tier on a 16-key C4 batch (uncontended: per-key latency)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/t3sq
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_WAIT_ANY -d gpurun_out/t3sq/p1 -o p1 --output-format csv -- python3 tools/t3_prof.py 65536 16 > gpurun_out/t3sq/p1.log 2>&1 || { tail -20 gpurun_out/t3sq/p1.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_VMEM SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM -d gpurun_out/t3sq/p2 -o p2 --output-format csv -- python3 tools/t3_prof.py 65536 16 > gpurun_out/t3sq/p2.log 2>&1 || { tail -20 gpurun_out/t3sq/p2.log; exit 1; }
echo done
