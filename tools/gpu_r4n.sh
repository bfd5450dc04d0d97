# Round 4: A/B of the WGL child-move adoption (default build against
# LC_WGL_ADOPT=0), alternating on one box: C2 and C4 WGL lines.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r4n
mkdir -p $O
for r in 1 2; do
  for v in adopt noadopt; do
    L=""; [ $v = noadopt ] && L=jepsen-etcd-demo_amd/lincheck/liblincheck_noadopt.so
    echo "== $v round $r $(date +%T)"
    LINCHECK_LIB_OVERRIDE=$L timeout -k 10 300 python -u bench.py --config C2 --algorithm wgl --steps 10 --warmup 2 --no-resident --no-c3 --no-cpu > $O/c2_${v}_$r.json 2> $O/c2_${v}_$r.err || { tail -5 $O/c2_${v}_$r.err; exit 1; }
    LINCHECK_LIB_OVERRIDE=$L timeout -k 10 300 python -u bench.py --config C4 --budget 65536 --algorithm wgl --steps 3 --warmup 1 --no-resident --no-cpu > $O/c4_${v}_$r.json 2> $O/c4_${v}_$r.err || { tail -5 $O/c4_${v}_$r.err; exit 1; }
    python3 -c "import json,sys; [print(f, round(json.loads(open(f).read().strip().splitlines()[-1])['ms_per_step'],3)) for f in sys.argv[1:]]" $O/c2_${v}_$r.json $O/c4_${v}_$r.json
  done
done
echo ALL_OK
