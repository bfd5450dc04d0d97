# Quick check: node tests + parity tests, C2 bench, T0 PMC traffic passes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/q
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_node.py tests/test_gpu_parity.py -m gpu -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { grep -E "FAILED|^E " $O/tests.log | head -20; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u bench.py --steps 50 --warmup 5 > $O/bench_c2.json 2> $O/bench_c2.err || { tail -5 $O/bench_c2.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_c2.json'));print('value',d['value'],'ms',d['ms_per_step'],'T0',d['tier0_ms'],'resident',d['resident']['ops_per_s'])"
PROF="--no-cpu --no-resident --no-probes"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/f -o f --output-format csv -- python3 bench.py --steps 5 --warmup 1 $PROF > $O/f.log 2>&1 || { tail -5 $O/f.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/w -o w --output-format csv -- python3 bench.py --steps 5 --warmup 1 $PROF > $O/w.log 2>&1 || { tail -5 $O/w.log; exit 1; }
python3 tools/pmc_bytes.py lattice $O/f/f_counter_collection.csv $O/w/w_counter_collection.csv C2 1048576 $O/pmc.json "quick" | cut -c1-300
python3 tools/pmc_bytes.py validate $O/f/f_counter_collection.csv $O/w/w_counter_collection.csv C2 1048576 $O/pmc_v.json "quick" | cut -c1-300
