# GPU suite (one pytest process, each test bounded) then a C2 bench line.
# usage: tools/gpu_check.sh [pytest -k expression]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/check
mkdir -p $O
K=${1:+-k "$1"}
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -x --timeout 300 --timeout-method thread $K > $O/tests.log 2>&1
rc=$?
grep -E "FAILED|ERROR" $O/tests.log | head -20
tail -2 $O/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 50 --warmup 5 > $O/bench_c2.json 2> $O/bench_c2.err || { tail -5 $O/bench_c2.err; exit 1; }
cut -c1-600 $O/bench_c2.json
echo ALL_OK
