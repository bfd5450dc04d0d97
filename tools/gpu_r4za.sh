# Round 4: A/B on one box -- the speculative walk's closure in three widths
# (base: four, five, six ops) against four (top3, LC_T0_TOP3=1: three live
# ops get their own body): C2, C5, the C3 shard; then the GPU suite.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r4za
mkdir -p $O
lib() { [ $1 = base ] && echo "" || echo jepsen-etcd-demo_amd/lincheck/liblincheck_$1.so; }
ms() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d.get('roofline') or {}; print(sys.argv[1], round(d['ms_per_step'],4), r.get('avg_launch_ms'))" $1; }
for r in 1 2; do
  for v in base top3; do
    echo "== $v round $r $(date +%T)"
    LINCHECK_LIB_OVERRIDE=$(lib $v) timeout -k 10 300 python -u bench.py --steps 50 --warmup 5 --no-cpu --no-c3 > $O/c2_${v}_$r.json 2> $O/c2_${v}_$r.err || { tail -5 $O/c2_${v}_$r.err; exit 1; }
    ms $O/c2_${v}_$r.json
    LINCHECK_LIB_OVERRIDE=$(lib $v) timeout -k 10 300 python -u bench.py --config C5 --steps 30 --warmup 3 --no-cpu > $O/c5_${v}_$r.json 2> $O/c5_${v}_$r.err || { tail -5 $O/c5_${v}_$r.err; exit 1; }
    ms $O/c5_${v}_$r.json
    LINCHECK_LIB_OVERRIDE=$(lib $v) timeout -k 10 300 python -u bench.py --config C3 --keys 12500 --steps 10 --warmup 2 --no-cpu > $O/c3s_${v}_$r.json 2> $O/c3s_${v}_$r.err || { tail -5 $O/c3s_${v}_$r.err; exit 1; }
    ms $O/c3s_${v}_$r.json
  done
done
echo "== tests $(date +%T)"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|^E " $O/tests.log | head -20; exit 1; }
tail -1 $O/tests.log
echo ALL_OK
