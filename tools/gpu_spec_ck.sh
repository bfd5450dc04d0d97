# Sweep of the speculative segments' checkpoint distances (LC_SPEC_CK1 /
# LC_SPEC_CK2, defaults 32 / 160) and segments per key on C2, pipelined step.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/specck
mkdir -p $O
run() {
  timeout -k 10 120 python -u bench.py --steps 100 --warmup 10 --no-cpu --no-resident --no-probes > $O/b.json 2> $O/b.err || { tail -5 $O/b.err; exit 1; }
  python -c "import json;d=json.load(open('$O/b.json'));print('$1', round(d['ms_per_step'],4), round(d['roofline']['avg_launch_ms'],4), d['d1_sync']['same_records'])"
}
for ck in ${SWEEP:-32:160 16:96 24:128 48:200 64:256 32:120 32:240}; do
  set -- ${ck/:/ }
  export LC_SPEC_CK1=$1 LC_SPEC_CK2=$2
  run "ck=$1/$2"
done
unset LC_SPEC_CK1 LC_SPEC_CK2
[ -z "$SWEEP" ] && for sg in 3 6; do export LC_SPEC_SEGS=$sg; run "segs=$sg"; done
echo ALL_OK
