# Register-tier A/B after a kernel change: C2 / C5 (default against the
# unsegmented tier), C3 shards of 12.5k and 25k keys and the whole C3 key space
# (speculative segments, now the default for large batches, against
# LC_PATH_SPEC_OFF = 0x4), then the GPU suite and the default bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/c3spec
mkdir -p $O
echo "== ab $(date +%T)"
timeout -k 10 300 python -u tools/spec_ab.py C2 1000 1000 default > $O/ab_c2.txt 2>&1 || { tail -5 $O/ab_c2.txt; exit 1; }
cat $O/ab_c2.txt
timeout -k 10 300 python -u tools/spec_ab.py C5 1000 1000 default > $O/ab_c5.txt 2>&1 || { tail -5 $O/ab_c5.txt; exit 1; }
cat $O/ab_c5.txt
for K in 12500 25000; do
timeout -k 10 300 python -u tools/spec_ab.py C3 $K 2000 default path_flags=0x4 > $O/ab_c3_$K.txt 2>&1 || { tail -5 $O/ab_c3_$K.txt; exit 1; }
cat $O/ab_c3_$K.txt
done
timeout -k 10 400 python -u tools/spec_ab.py C3 100000 2000 default path_flags=0x4 > $O/ab_c3_100k.txt 2>&1 || { tail -5 $O/ab_c3_100k.txt; exit 1; }
cat $O/ab_c3_100k.txt
if [ -z "$NOTEST" ]; then
echo "== tests $(date +%T)"
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|^E " $O/tests.log | head -20; exit 1; }
tail -1 $O/tests.log
fi
echo "== bench $(date +%T)"
timeout -k 10 400 python -u bench.py --steps 50 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
cut -c1-300 $O/bench.json
python3 -c "import json;d=json.loads(open('$O/bench.json').read());print(json.dumps(d['c3_strong']))"
echo ALL_OK
