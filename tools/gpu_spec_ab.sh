# A/B of speculative-segment variants: stamps of each variant library, tests, bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/specab
mkdir -p $O
for v in ${VARIANTS:-specst specclosed}; do
  LINCHECK_LIB_OVERRIDE=$PWD/jepsen-etcd-demo_amd/lincheck/liblincheck_$v.so timeout -k 10 200 python tools/spec_stamps.py > $O/stamps_$v.txt 2>&1 || { tail -5 $O/stamps_$v.txt; exit 1; }
  echo "== $v"; head -9 $O/stamps_$v.txt | tail -8
done
timeout -k 10 300 python -m pytest tests/test_gpu_spec.py -x -q --timeout 120 > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
LC_SPEC=1 timeout -k 10 300 python bench.py --steps 40 --warmup 5 --no-cpu --no-probes > $O/b.json 2> $O/b.err || { tail -5 $O/b.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/b.json'));print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['resident']['ms_per_step'])"
