# Round 4: WGL whole child move only when R's op has the earliest legal :invoke
# -- the WGL GPU tests, the C2 / C4 WGL lines.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r4m
mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
step tests
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -k "wgl or WGL or competition" --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|^E " $O/tests.log | head -20; exit 1; }
tail -1 $O/tests.log
step bench_c2_wgl
timeout -k 10 400 python -u bench.py --config C2 --algorithm wgl --steps 10 --warmup 2 --no-resident --no-c3 > $O/bench_c2_wgl.json 2> $O/bench_c2_wgl.err || { tail -5 $O/bench_c2_wgl.err; exit 1; }
cut -c1-200 $O/bench_c2_wgl.json
step bench_c4_wgl
timeout -k 10 400 python -u bench.py --config C4 --budget 65536 --algorithm wgl --steps 3 --warmup 1 --no-resident --no-cpu > $O/bench_c4_wgl.json 2> $O/bench_c4_wgl.err || { tail -5 $O/bench_c4_wgl.err; exit 1; }
cut -c1-200 $O/bench_c4_wgl.json
echo ALL_OK
