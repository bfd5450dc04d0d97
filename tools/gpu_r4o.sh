# Round 4: A/B on one box -- WGL child-move adoption (default, LC_WGL_ADOPT=0,
# =2: only when R's op has the earliest legal :invoke) on C2 / C4 WGL; the
# lane-phase closure loop without a trip counter (LC_T0_SWEEP_DO=1) on C2 / C5.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r4o
mkdir -p $O
lib() { [ $1 = base ] && echo "" || echo jepsen-etcd-demo_amd/lincheck/liblincheck_$1.so; }
ms() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d.get('roofline') or {}; print(sys.argv[1], round(d['ms_per_step'],4), r.get('kernel'), r.get('avg_launch_ms'))" $1; }
for r in 1 2; do
  for v in base sweepdo; do
    echo "== linear $v round $r $(date +%T)"
    LINCHECK_LIB_OVERRIDE=$(lib $v) timeout -k 10 300 python -u bench.py --steps 50 --warmup 5 --no-cpu --no-c3 > $O/c2_${v}_$r.json 2> $O/c2_${v}_$r.err || { tail -5 $O/c2_${v}_$r.err; exit 1; }
    ms $O/c2_${v}_$r.json
    LINCHECK_LIB_OVERRIDE=$(lib $v) timeout -k 10 300 python -u bench.py --config C5 --steps 30 --warmup 3 --no-cpu > $O/c5_${v}_$r.json 2> $O/c5_${v}_$r.err || { tail -5 $O/c5_${v}_$r.err; exit 1; }
    ms $O/c5_${v}_$r.json
  done
done
for r in 1 2; do
  for v in base noadopt adopt2; do
    echo "== wgl $v round $r $(date +%T)"
    LINCHECK_LIB_OVERRIDE=$(lib $v) timeout -k 10 300 python -u bench.py --config C2 --algorithm wgl --steps 10 --warmup 2 --no-resident --no-c3 --no-cpu > $O/w2_${v}_$r.json 2> $O/w2_${v}_$r.err || { tail -5 $O/w2_${v}_$r.err; exit 1; }
    ms $O/w2_${v}_$r.json
    LINCHECK_LIB_OVERRIDE=$(lib $v) timeout -k 10 300 python -u bench.py --config C4 --budget 65536 --algorithm wgl --steps 3 --warmup 1 --no-resident --no-cpu > $O/w4_${v}_$r.json 2> $O/w4_${v}_$r.err || { tail -5 $O/w4_${v}_$r.err; exit 1; }
    ms $O/w4_${v}_$r.json
  done
done
echo ALL_OK
