# C3 per-GPU shard (12,500 keys x 2,000 ops): bench line and rocprofv3 kernel stats.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/c3s
mkdir -p $O
B="python3 bench.py --config C3 --keys 12500 --steps 10 --warmup 2 --no-cpu --no-probes"
timeout -k 10 300 $B > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
cut -c1-300 $O/bench.json; grep -o '"tier0_ms": [0-9.]*\|"resident": {[^}]*}' $O/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- $B --no-resident > $O/kt.log 2>&1 || { tail -20 $O/kt.log; exit 1; }
f=$(find $O/kt -name "*kernel_stats.csv" | head -1); cut -d, -f1-8 "$f" | head -12
echo ALL_OK
