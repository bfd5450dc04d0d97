# (Record of round 6's cooperative-T3L runs, commit 141027e; that build was reverted after them: profiles/r06_t3l_coop.txt.)
# Round 6: T3L cooperation -- is the slowdown the helpers' polling?  Helpers
# poll but no block posts (LC_T3L_COOP_MAX=1) against no cooperation.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6y2; mkdir -p $O
L=$PWD/jepsen-etcd-demo_amd/lincheck
for v in pollonly nocoop pollonly; do
  LINCHECK_LIB_OVERRIDE=$L/liblincheck_$v.so timeout -k 10 200 python -u bench.py --config C4 --budget 65536 --steps 3 --warmup 1 --no-cpu --no-resident --no-probes --no-c3 > $O/c4_$v.json 2> $O/c4_$v.err || { tail -5 $O/c4_$v.err; exit 1; }
  python -c "import json,sys; d=json.loads(open('$O/c4_$v.json').read().strip().splitlines()[-1]); print('$v', 'ms', round(d['ms_per_step'],3), 't3', d.get('tier3_ms'), d['verdicts'])"
done
