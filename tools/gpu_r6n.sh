# Round 6: the block set-up at issue priority 3 (LC_SPEC_CUT_PRIO=1 build)
# against 0 (default), with the overlapped TOP / verifying runs.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6n; mkdir -p $O
for c in C2 C5; do for sd in "" 11 15; do
  SEED=$sd timeout -k 10 200 python -u tools/spec_ab.py $c 1000 1000 default > $O/base_${c}_$sd.txt 2>&1 || { tail -5 $O/base_${c}_$sd.txt; exit 1; }
  SEED=$sd LINCHECK_LIB_OVERRIDE=$PWD/jepsen-etcd-demo_amd/lincheck/liblincheck_cutprio.so timeout -k 10 200 python -u tools/spec_ab.py $c 1000 1000 default > $O/prio_${c}_$sd.txt 2>&1 || { tail -5 $O/prio_${c}_$sd.txt; exit 1; }
  echo "$c seed ${sd:-default}: prio0 $(grep -o 'median [0-9.]*' $O/base_${c}_$sd.txt) / prio3 $(grep -o 'median [0-9.]*' $O/prio_${c}_$sd.txt)"
done; done
