# Round 6: the speculative segments' first checkpoint distance (lc_opts.spec_ck)
# on C2 and C5, records checked equal across settings.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6f; mkdir -p $O
for c in C2 C5; do
  timeout -k 10 300 python -u tools/spec_ab.py $c 1000 1000 default spec_ck=0x790011 spec_ck=0x790019 spec_ck=0x790009 spec_ck=0x990011 default > $O/ck_$c.txt 2>&1 || { tail -5 $O/ck_$c.txt; exit 1; }
  cat $O/ck_$c.txt
done
