# A/B of T3 builds on the C4 batch (arg: variant names, "" = product library)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
for v in "" u2 u8; do
  L=""; [ -n "$v" ] && L=$GRAFT_REPO_ROOT/jepsen-etcd-demo_amd/lincheck/liblincheck_$v.so
  for b in 65536 1048576; do
    LINCHECK_LIB_OVERRIDE=$L timeout -k 10 200 python -u tools/t3_prof.py $b > gpurun_out/ab_$v_$b.log 2>&1 || { echo "FAIL $v $b"; tail -5 gpurun_out/ab_$v_$b.log; exit 1; }
    echo "lib=${v:-product} budget=$b $(tail -1 gpurun_out/ab_$v_$b.log)"
  done
done
