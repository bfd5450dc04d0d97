# A/B of the D-1 step on C2: events DMA'd (default) vs read in place from
# page-locked host memory (LC_ZEROCOPY=1), plus the LC_TIMING breakdown.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/zc
mkdir -p $O
for zc in 0 1 0 1; do
  LC_ZEROCOPY=$zc timeout -k 10 200 python -u bench.py --steps 40 --warmup 5 --no-cpu --no-probes > $O/bench_zc$zc.json 2> $O/bench_zc$zc.err || { tail -5 $O/bench_zc$zc.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/bench_zc$zc.json').read().splitlines()[-1]);print('zc=$zc', round(d['value']/1e9,3),'Gops/s', round(d['ms_per_step'],4),'ms', 'T0', round(d['tier0_ms'],4), 'res', round(d['resident']['ms_per_step'],4), d['parity_vs_oracle'])"
done
LC_TIMING=1 timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-cpu --no-probes --no-resident > $O/timing0.json 2> $O/timing0.err || exit 1
grep lc_check_node $O/timing0.err | tail -4
LC_ZEROCOPY=1 LC_TIMING=1 timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-cpu --no-probes --no-resident > $O/timing1.json 2> $O/timing1.err || exit 1
grep lc_check_node $O/timing1.err | tail -4
echo ALL_OK
for zc in 0 1; do
  LC_ZEROCOPY=$zc timeout -k 10 300 python -u bench.py --config C3 --keys 20000 --steps 5 --warmup 1 --no-cpu --no-probes --no-resident > $O/c3_zc$zc.json 2> $O/c3_zc$zc.err || { tail -5 $O/c3_zc$zc.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/c3_zc$zc.json').read().splitlines()[-1]);print('C3-20k zc=$zc', round(d['value']/1e9,3),'Gops/s', round(d['ms_per_step'],3),'ms T0', round(d['tier0_ms'],3))"
done
echo C3_OK
