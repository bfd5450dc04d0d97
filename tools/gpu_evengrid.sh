# A/B: T0 grid sized to whole rounds of keys (default) or the full 16 waves
# per CU (LC_T0_FULLGRID=1), on the per-rank C3 shards of N = 8, 4, 2 and 1.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/evengrid
mkdir -p $O
for k in 12500 25000 50000; do
  for v in even full; do
    if [ $v = full ]; then export LC_T0_FULLGRID=1; else unset LC_T0_FULLGRID; fi
    timeout -k 10 300 python -u bench.py --config C3 --keys $k --steps 5 --warmup 1 --no-cpu --no-probes > $O/b_${k}_$v.json 2> $O/b_${k}_$v.err || { tail -5 $O/b_${k}_$v.err; exit 1; }
    python -c "import json;d=json.load(open('$O/b_${k}_$v.json'));print($k, '$v', d['value'], d['ms_per_step'], d['resident']['ms_per_step'], d['d1_sync']['same_records'], d['resident']['same_records_as_d1'])"
  done
done
echo ALL_OK
