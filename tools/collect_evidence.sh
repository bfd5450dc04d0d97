# gpurun_out/r$R (tools/gpu_evidence.sh) -> profiles/r0$R_*: kernel-stats
# summaries, traffic / SQ summaries over whole launches (tools/
# profile_summary.py), bench lines and the GPU suite's summary.
#   R=5 bash tools/collect_evidence.sh
set -e
cd "$(dirname "$0")/.."
R=${R:-5}
O=${O:-gpurun_out/r$R}
P=profiles
T=$(printf "r%02d" $R)
csv() { find "$O/prof/$1" -name "$2" 2>/dev/null | head -1; }
for n in c2 c5 c3s c4 c4wgl c2wgl; do
  f=$(csv kt_$n '*kernel_stats.csv'); [ -n "$f" ] && cp "$f" $P/${T}_${n}_kernel_stats.csv
done
pmc() {  # name kernel workload keys budget algorithm
  local n=$1 k=$2 w=$3 keys=$4 b=$5 alg=$6
  local fc=$(csv f_$n '*counter_collection.csv') wc=$(csv w_$n '*counter_collection.csv')
  local s1=$(csv sq1_$n '*counter_collection.csv') s2=$(csv sq2_$n '*counter_collection.csv')
  local cmd="rocprofv3 --pmc <counters> -- python3 bench.py (tools/gpu_evidence.sh part $n, R=$R)"
  [ -n "$fc" ] && [ -n "$wc" ] && python3 tools/profile_summary.py bytes --kernel "$k" --workload $w --keys $keys \
      --budget $b --round $R --algorithm $alg --cmd "$cmd" --out $P/${T}_${n}_pmc.json "$fc" "$wc"
  [ -n "$s1" ] && [ -n "$s2" ] && python3 tools/profile_summary.py sq --kernel "$k" --workload $w --keys $keys \
      --budget $b --round $R --algorithm $alg --cmd "$cmd" --out $P/${T}_${n}_sq.json "$s1" "$s2"
  return 0
}
# whole-launch kernel times from the traces (the stats CSV mixes launch sizes)
tr() {  # name kernel workload keys budget algorithm
  local t=$(csv kt_$1 '*kernel_trace.csv')
  [ -n "$t" ] && python3 tools/profile_summary.py trace --kernel "$2" --workload $3 --keys $4 --budget $5 --round $R \
      --algorithm $6 --cmd "rocprofv3 --kernel-trace --stats -- python3 bench.py (tools/gpu_evidence.sh part $1)" \
      --out $P/${T}_$1_trace.json "$t"
  return 0
}
tr c3s "k_spec<" C3 12500 1048576 linear
tr c4wgl "k_wgl" C4 256 65536 wgl
tr c2wgl "k_wgl" C2 1000 1048576 wgl
pmc c2 "k_spec<" C2 1000 1048576 linear
pmc c3s "k_spec<" C3 12500 1048576 linear
pmc c4 "k_search_layers" C4 256 65536 linear
pmc c4wgl "k_wgl" C4 256 65536 wgl
pmc c2wgl "k_wgl" C2 1000 1048576 wgl
for b in c2 c5 c3s c4 c4_wgl c4_comp c2_wgl c5_jepsen c4_wgl24; do
  [ -f "$O/bench_$b.json" ] && tail -1 "$O/bench_$b.json" > $P/${T}_${b}_bench.json
done
[ -f "$O/tests.log" ] && { grep -E "passed|failed" "$O/tests.log" | tail -1 > $P/${T}_gpu_tests_summary.txt; }
ls $P | grep "^$T" || true
