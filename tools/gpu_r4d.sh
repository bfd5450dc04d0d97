# Round 4, k_spec lane-phase sweep masks (LC_SPEC_PMASK) A/B: the spec /
# parity GPU tests on the new build, then C2 and C5 bench lines and kernel
# traces for the new build and the PMASK=0 variant (LINCHECK_LIB_OVERRIDE,
# A/B only), alternating.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r4d
mkdir -p $O/prof
step() { echo "== $1 $(date +%T)"; }
step tests
timeout -k 10 600 python -u -m pytest tests/test_gpu_spec.py tests/test_gpu_parity.py tests/test_gpu_events16.py -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|^E " $O/tests.log | head -20; exit 1; }
tail -1 $O/tests.log
for rep in 1 2; do
for v in new pm0; do
  if [ $v = pm0 ]; then export LINCHECK_LIB_OVERRIDE=jepsen-etcd-demo_amd/lincheck/liblincheck_pm0.so; else unset LINCHECK_LIB_OVERRIDE; fi
  step bench_c2_${v}_$rep
  timeout -k 10 300 python -u bench.py --config C2 --steps 50 --warmup 5 --no-resident --no-c3 --no-cpu --no-probes > $O/c2_${v}_$rep.json 2> $O/c2_${v}_$rep.err || { tail -5 $O/c2_${v}_$rep.err; exit 1; }
  cut -c1-200 $O/c2_${v}_$rep.json
  step bench_c5_${v}_$rep
  timeout -k 10 300 python -u bench.py --config C5 --steps 50 --warmup 5 --no-resident --no-c3 --no-cpu --no-probes > $O/c5_${v}_$rep.json 2> $O/c5_${v}_$rep.err || { tail -5 $O/c5_${v}_$rep.err; exit 1; }
done
done
for v in new pm0; do
  if [ $v = pm0 ]; then export LINCHECK_LIB_OVERRIDE=jepsen-etcd-demo_amd/lincheck/liblincheck_pm0.so; else unset LINCHECK_LIB_OVERRIDE; fi
  step prof_c2_$v
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof/c2_$v -o c2 --output-format csv -- python3 bench.py --config C2 --steps 50 --warmup 5 --no-resident --no-c3 --no-cpu --no-probes > $O/prof/c2_$v.log 2>&1 || { tail -5 $O/prof/c2_$v.log; exit 1; }
done
echo ALL_OK
