# Round 6: cuts at equal estimated cost (LC_PATH_SPEC_COST, 0x100) against
# equal event counts, on the overlapped build.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6p; mkdir -p $O
for c in C2 C5; do for sd in "" 11 15; do
  SEED=$sd timeout -k 10 200 python -u tools/spec_ab.py $c 1000 1000 default path_flags=0x100 > $O/${c}_$sd.txt 2>&1 || { tail -5 $O/${c}_$sd.txt; exit 1; }
  echo "$c seed ${sd:-default}: $(grep -o 'median [0-9.]*' $O/${c}_$sd.txt | tr '\n' ' ') (events / cost)"
done; done
