# A/B of library builds on one box (replaces round 4's one-off gpu_r4*.sh).
# VARIANTS: "base" = the product build, NAME = lincheck/liblincheck_NAME.so
# (make variant NAME=... VFLAGS=...); WORKLOADS: c2 c5 c3s c4 c2wgl c4wgl;
# ROUNDS: repetitions (interleaved, so a box's drift hits every variant).
# Prints per run: ms per step, the dominant kernel, its average launch ms.
#   VARIANTS="base foo" WORKLOADS="c2 c5" ROUNDS=2 TAG=ab1 bash tools/gpu_ab.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-ab}
mkdir -p $O
lib() { [ $1 = base ] && echo "" || echo $PWD/jepsen-etcd-demo_amd/lincheck/liblincheck_$1.so; }
args() {
  case $1 in
  c2) echo "--steps 50 --warmup 5 --no-cpu --no-c3" ;;
  c5) echo "--config C5 --steps 30 --warmup 3 --no-cpu" ;;
  c3s) echo "--config C3 --keys 12500 --steps 10 --warmup 2 --no-cpu" ;;
  c4) echo "--config C4 --budget 65536 --steps 3 --warmup 1 --no-cpu --no-probes" ;;
  c2wgl) echo "--config C2 --algorithm wgl --steps 10 --warmup 2 --no-resident --no-c3 --no-cpu" ;;
  c4wgl) echo "--config C4 --budget 65536 --algorithm wgl --steps 3 --warmup 1 --no-resident --no-cpu" ;;
  *) echo "unknown workload $1" >&2; exit 2 ;;
  esac
}
ms() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d.get('roofline') or {}; print(sys.argv[1], round(d['ms_per_step'],4), r.get('kernel'), r.get('avg_launch_ms'), d.get('verdicts'))" $1; }
for r in $(seq 1 ${ROUNDS:-1}); do
  for w in ${WORKLOADS:-c2}; do
    for v in ${VARIANTS:-base}; do
      echo "== $w $v round $r $(date +%T)"
      LINCHECK_LIB_OVERRIDE=$(lib $v) timeout -k 10 ${LIMIT:-300} python -u bench.py $(args $w) ${EXTRA:-} > $O/${w}_${v}_$r.json 2> $O/${w}_${v}_$r.err || { tail -5 $O/${w}_${v}_$r.err; exit 1; }
      ms $O/${w}_${v}_$r.json
    done
  done
done
echo ALL_OK
