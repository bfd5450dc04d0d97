# C2 sweep over segments per key (speculative segments).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/spec
mkdir -p $O
run() {  # label, env...
  local lab=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --steps 40 --warmup 5 --no-cpu --no-probes > $O/sw_$lab.json 2> $O/sw_$lab.err || { tail -5 $O/sw_$lab.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/sw_$lab.json'));print('$lab', round(d['value']/1e9,3), round(d['ms_per_step'],4), round(d['roofline']['avg_launch_ms'],4), round(d['resident']['ms_per_step'],4))"
}
for s in ${SEGS:-3 4 6 8}; do run s$s LC_SPEC=1 LC_SPEC_SEGS=$s; done
