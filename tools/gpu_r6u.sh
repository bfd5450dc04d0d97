# Round 6: three checkpoints per TOP run (LC_SPEC_NCK=3: ck1 / 4, ck1, ck2)
# against two on the overlapped build, where a segment's verifying run starts
# right after the previous segment's TOP walk (often the block's last walk).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6u; mkdir -p $O
for c in C2 C5; do for sd in "" 11 15; do
  SEED=$sd timeout -k 10 200 python -u tools/spec_ab.py $c 1000 1000 default > $O/two_${c}_$sd.txt 2>&1 || { tail -5 $O/two_${c}_$sd.txt; exit 1; }
  SEED=$sd LINCHECK_LIB_OVERRIDE=$PWD/jepsen-etcd-demo_amd/lincheck/liblincheck_ck3.so timeout -k 10 300 python -u tools/spec_ab.py $c 1000 1000 default spec_ck=0x790031 spec_ck=0x790041 > $O/three_${c}_$sd.txt 2>&1 || { tail -5 $O/three_${c}_$sd.txt; exit 1; }
  echo "$c seed ${sd:-default}: two (32,120) $(grep -o 'median [0-9.]*' $O/two_${c}_$sd.txt) / three (8,32,120) (12,48,120) (16,64,120) $(grep -o 'median [0-9.]*' $O/three_${c}_$sd.txt | tr '\n' ' ')"
done; done
