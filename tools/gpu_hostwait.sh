# A/B: the pipelined step's search waiting for its upload on the device
# (cross-stream event) or on the host (no device-side wait).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/hostwait
mkdir -p $O
for v in dev host dev host; do
  if [ $v = host ]; then export LC_PIPE_HOSTWAIT=1; else unset LC_PIPE_HOSTWAIT; fi
  timeout -k 10 300 python -u bench.py --steps 200 --warmup 10 --no-cpu --no-resident --no-probes > $O/bench_$v.json 2> $O/bench_$v.err || { tail -5 $O/bench_$v.err; exit 1; }
  python -c "import json;d=json.load(open('$O/bench_$v.json'));print('$v', d['value'], d['ms_per_step'], d['d1_sync']['same_records'])"
done
echo ALL_OK
