# Round-4 evidence -> profiles/: the rocprofv3 kernel-stats summaries, the
# FETCH_SIZE / WRITE_SIZE traffic and SQ summaries (tagged round 4, the only
# ones bench.py quotes this round) and the bench lines, from the
# gpurun_out/r4 tree tools/gpu_evidence_r4.sh leaves.
set -e
cd "$(dirname "$0")/.."
O=${1:-gpurun_out/r4}
P=profiles
csv() { find "$O/prof/$1" -name "$2" | head -1; }
for n in c2 c3s c4 c4wgl c2wgl; do
  f=$(csv kt_$n '*kernel_stats.csv'); [ -n "$f" ] && cp "$f" $P/r04_${n}_kernel_stats.csv
done
pmc() {  # name kernel workload budget
  local n=$1 k=$2 w=$3 b=$4
  local fc=$(csv f_$n '*counter_collection.csv') wc=$(csv w_$n '*counter_collection.csv')
  local s1=$(csv sq1_$n '*counter_collection.csv') s2=$(csv sq2_$n '*counter_collection.csv')
  [ -n "$fc" ] && [ -n "$wc" ] && python3 tools/pmc_bytes.py "$k" "$fc" "$wc" "$w" "$b" $P/r04_${n}_pmc.json \
      "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE -- python3 bench.py (tools/gpu_evidence_r4.sh pmc $n)" 4 > /dev/null
  [ -n "$s1" ] && [ -n "$s2" ] && LC_ROUND=4 python3 tools/sq_summary.py "$k" "$w" "$b" $P/r04_${n}_sq.json \
      "rocprofv3 --pmc SQ_* -- python3 bench.py (tools/gpu_evidence_r4.sh pmc $n)" "$s1" "$s2" > /dev/null
  return 0
}
pmc c2 "k_spec<4, 4, true, false>" C2 1048576
pmc c3s "k_spec<2, 2, true, false>" C3 1048576
pmc c4 "k_search_layers" C4 65536
for b in c2 c5 c3s c4 c4_wgl c4_comp c2_wgl c5_jepsen; do
  [ -f "$O/bench_$b.json" ] && tail -1 "$O/bench_$b.json" > $P/r04_${b}_bench.json
done
[ -f "$O/tests.log" ] && { grep -E "PASSED|FAILED|ERROR|passed|failed" "$O/tests.log" | tail -3 > $P/r04_gpu_tests_summary.txt; }
ls -la $P | grep r04
