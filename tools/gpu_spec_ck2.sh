# Finer sweep of the second checkpoint distance on C2 and C5 (pipelined step).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/specck2
mkdir -p $O
run() {
  timeout -k 10 120 python -u bench.py --config $2 --steps 100 --warmup 10 --no-cpu --no-resident --no-probes > $O/b.json 2> $O/b.err || { tail -5 $O/b.err; exit 1; }
  python -c "import json;d=json.load(open('$O/b.json'));print('$1 $2', round(d['ms_per_step'],4), round(d['roofline']['avg_launch_ms'],4), d['d1_sync']['same_records'])"
}
for cfg in C2 C5; do
  for ck in ${SWEEP:-32:160 32:120 32:100 32:110 32:130 32:140 24:120 40:120 32:160 32:120}; do
    set -- ${ck/:/ }
    export LC_SPEC_CK1=$1 LC_SPEC_CK2=$2
    run "ck=$1/$2" $cfg
  done
done
echo ALL_OK
