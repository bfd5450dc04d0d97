# GPU suite + D-1 timing breakdown + C2 bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/q2
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|^E " $O/tests.log | head -30; exit 1; }
tail -1 $O/tests.log
timeout -k 10 120 python tools/node_timing.py 2>&1 | tail -3
timeout -k 10 300 python -u bench.py --steps 50 --warmup 5 --no-cpu > $O/b.json 2> $O/b.err || { tail -5 $O/b.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/b.json'));print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['resident']['ms_per_step'])"
