# (Record of round 6's cooperative-T3L runs, commit 141027e; that build was reverted after them: profiles/r06_t3l_coop.txt.)
# Round 6: T3L cooperating blocks (LC_T3L_COOP) -- the layered tier's GPU
# tests, then C4 at 2^16 with and without cooperation (T3L kernel time).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6w; mkdir -p $O
L=$PWD/jepsen-etcd-demo_amd/lincheck
timeout -k 10 300 python -u -m pytest tests/test_gpu_layers.py -x -v --timeout 120 --timeout-method thread > $O/layers.log 2>&1 || { tail -30 $O/layers.log; exit 1; }
tail -3 $O/layers.log
for v in coop nocoop coop nocoop; do
  if [ $v = coop ]; then unset LINCHECK_LIB_OVERRIDE; else export LINCHECK_LIB_OVERRIDE=$L/liblincheck_nocoop.so; fi
  timeout -k 10 200 python -u bench.py --config C4 --budget 65536 --steps 3 --warmup 1 --no-cpu --no-resident --no-probes --no-c3 > $O/c4_$v.json 2> $O/c4_$v.err || { tail -5 $O/c4_$v.err; exit 1; }
  python -c "import json,sys; d=json.loads(open('$O/c4_$v.json').read().strip().splitlines()[-1]); print('$v', 'ms', round(d['ms_per_step'],3), 't3', d.get('tier3_ms'), d['verdicts'], d.get('parity_vs_oracle'))"
done
unset LINCHECK_LIB_OVERRIDE


