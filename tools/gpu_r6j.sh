# Round 6: the block set-up (staging, validation, cuts) at issue priority 3
# (default build) against priority 0 (LC_SPEC_CUT_PRIO=0 build), on C2 and C5
# and two other seeds of each; records equal.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6j; mkdir -p $O
for c in C2 C5; do for sd in "" 11 15; do
  SEED=$sd timeout -k 10 200 python -u tools/spec_ab.py $c 1000 1000 default > $O/new_${c}_$sd.txt 2>&1 || { tail -5 $O/new_${c}_$sd.txt; exit 1; }
  SEED=$sd LINCHECK_LIB_OVERRIDE=$PWD/jepsen-etcd-demo_amd/lincheck/liblincheck_nocutprio.so timeout -k 10 200 python -u tools/spec_ab.py $c 1000 1000 default > $O/old_${c}_$sd.txt 2>&1 || { tail -5 $O/old_${c}_$sd.txt; exit 1; }
  echo "$c seed ${sd:-default}: new $(grep -o 'median [0-9.]*' $O/new_${c}_$sd.txt) / old $(grep -o 'median [0-9.]*' $O/old_${c}_$sd.txt)"
done; done
