# Round 4, final lines: PART=B of tools/gpu_evidence_r4.sh (C4 linear / WGL /
# competition, C2 WGL, C5 --jepsen, WGL phase cycles), then the C2 default and
# C3-shard lines again, whose traffic / issue fields now come from the profiles
# PART=A left (collected into profiles/ before this call).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
SKIP_TESTS=1 PART=B bash tools/gpu_evidence_r4.sh || exit 1
O=gpurun_out/r4
echo "== bench_c2 (final) $(date +%T)"
timeout -k 10 400 python -u bench.py --steps 50 --warmup 5 > $O/bench_c2.json 2> $O/bench_c2.err || { tail -5 $O/bench_c2.err; exit 1; }
cut -c1-200 $O/bench_c2.json
echo "== bench_c3_shard (final) $(date +%T)"
timeout -k 10 300 python -u bench.py --config C3 --keys 12500 --steps 10 --warmup 2 --no-cpu > $O/bench_c3s.json 2> $O/bench_c3s.err || { tail -5 $O/bench_c3s.err; exit 1; }
cut -c1-200 $O/bench_c3s.json
echo ALL_OK
