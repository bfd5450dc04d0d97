# Round 6: 4 against 8 segments per key over several seeds of the C2 and C5
# shapes (is C5's loss at 8 the anomalies or the instance?).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6h; mkdir -p $O
for c in C2 C5; do for sd in 11 12 13 14 15 16; do
  SEED=$sd timeout -k 10 200 python -u tools/spec_ab.py $c 1000 1000 spec_segs=4 spec_segs=8 > $O/s_${c}_$sd.txt 2>&1 || { tail -5 $O/s_${c}_$sd.txt; exit 1; }
  echo "seed $sd"; cat $O/s_${c}_$sd.txt
done; done
