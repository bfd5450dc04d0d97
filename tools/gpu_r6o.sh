# Round 6: the overlapped verifying runs at issue priority 2 or 3
# (LC_SPEC_VER_PRIO builds) against 0 (default).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6o; mkdir -p $O
L=$PWD/jepsen-etcd-demo_amd/lincheck
for c in C2 C5; do for sd in "" 11 15; do
  for v in base vp2 vp3; do
    if [ $v = base ]; then unset LINCHECK_LIB_OVERRIDE; else export LINCHECK_LIB_OVERRIDE=$L/liblincheck_$v.so; fi
    SEED=$sd timeout -k 10 200 python -u tools/spec_ab.py $c 1000 1000 default > $O/${v}_${c}_$sd.txt 2>&1 || { tail -5 $O/${v}_${c}_$sd.txt; exit 1; }
  done
  unset LINCHECK_LIB_OVERRIDE
  echo "$c seed ${sd:-default}: prio0 $(grep -o 'median [0-9.]*' $O/base_${c}_$sd.txt) / prio2 $(grep -o 'median [0-9.]*' $O/vp2_${c}_$sd.txt) / prio3 $(grep -o 'median [0-9.]*' $O/vp3_${c}_$sd.txt)"
done; done
