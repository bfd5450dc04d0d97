# PMC passes over the HBM tier on the C4 batch (one counter group per run).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/t3pmc
i=0
for ctr in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_ATOMIC_sum TCC_ATOMIC_sum"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $ctr -d gpurun_out/t3pmc/p$i -o p$i --output-format csv -- python3 tools/t3_prof.py 65536 > gpurun_out/t3pmc/p$i.log 2>&1 || { echo "PASS $i ($ctr) FAILED"; tail -5 gpurun_out/t3pmc/p$i.log; }
done
ls -R gpurun_out/t3pmc | head -30
