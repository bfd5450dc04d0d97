# Round 4: T3L sizing, second pass (C4 at 2^16): the S' table at 1.5x (TSB 2)
# and 2x (TSB 1) its bound, TSB 2 with TSA 3 or FILL 5, against the defaults.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r4zc
mkdir -p $O
lib() { [ $1 = base ] && echo "" || echo jepsen-etcd-demo_amd/lincheck/liblincheck_$1.so; }
ms() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d.get('roofline') or {}; print(sys.argv[1], round(d['ms_per_step'],4), r.get('avg_launch_ms'), d.get('parity_vs_oracle'))" $1; }
for r in 1 2; do
  for v in base tsb2 tsb1 tsb2a3 tsb2f5; do
    LINCHECK_LIB_OVERRIDE=$(lib $v) timeout -k 10 300 python -u bench.py --config C4 --budget 65536 --steps 3 --warmup 1 --no-cpu > $O/c4_${v}_$r.json 2> $O/c4_${v}_$r.err || { tail -5 $O/c4_${v}_$r.err; exit 1; }
    ms $O/c4_${v}_$r.json
  done
done
echo ALL_OK
