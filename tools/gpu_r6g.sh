# Round 6: three checkpoints per TOP run (an early one at ck1 / 4; the
# LC_SPEC_NCK=3 build) against two, on C2 and C5; records equal across settings.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6g; mkdir -p $O
for c in C2 C5; do
  timeout -k 10 300 python -u tools/spec_ab.py $c 1000 1000 default > $O/two_$c.txt 2>&1 || { tail -5 $O/two_$c.txt; exit 1; }
  LINCHECK_LIB_OVERRIDE=$PWD/jepsen-etcd-demo_amd/lincheck/liblincheck_ck3.so timeout -k 10 300 python -u tools/spec_ab.py $c 1000 1000 default spec_ck=0x790019 spec_ck=0x790031 spec_ck=0x790029 > $O/three_$c.txt 2>&1 || { tail -5 $O/three_$c.txt; exit 1; }
  cat $O/two_$c.txt $O/three_$c.txt
done
