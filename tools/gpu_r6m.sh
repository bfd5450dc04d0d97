# Round 6: TOP walks and verifying runs overlapped in k_spec (LC_SPEC_OVERLAP,
# the default build) -- the register-tier GPU tests, then A/B against the
# barrier-separated phases (LC_SPEC_OVERLAP=0 build) on C2 / C5 and other seeds.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6m; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_spec.py tests/test_gpu_segments.py tests/test_gpu_parity.py tests/test_gpu_events16.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for c in C2 C5; do for sd in "" 11 15; do
  SEED=$sd timeout -k 10 200 python -u tools/spec_ab.py $c 1000 1000 default > $O/new_${c}_$sd.txt 2>&1 || { tail -5 $O/new_${c}_$sd.txt; exit 1; }
  SEED=$sd LINCHECK_LIB_OVERRIDE=$PWD/jepsen-etcd-demo_amd/lincheck/liblincheck_nooverlap.so timeout -k 10 200 python -u tools/spec_ab.py $c 1000 1000 default > $O/old_${c}_$sd.txt 2>&1 || { tail -5 $O/old_${c}_$sd.txt; exit 1; }
  echo "$c seed ${sd:-default}: overlap $(grep -o 'median [0-9.]*' $O/new_${c}_$sd.txt) $(grep -o 'pipelined [0-9.]*' $O/new_${c}_$sd.txt) / barrier $(grep -o 'median [0-9.]*' $O/old_${c}_$sd.txt) $(grep -o 'pipelined [0-9.]*' $O/old_${c}_$sd.txt)"
done; done
timeout -k 10 200 python -u tools/spec_ab.py C3 12500 2000 default > $O/new_c3.txt 2>&1 || { tail -5 $O/new_c3.txt; exit 1; }
LINCHECK_LIB_OVERRIDE=$PWD/jepsen-etcd-demo_amd/lincheck/liblincheck_nooverlap.so timeout -k 10 200 python -u tools/spec_ab.py C3 12500 2000 default > $O/old_c3.txt 2>&1 || { tail -5 $O/old_c3.txt; exit 1; }
echo "C3 shard: overlap $(grep -o 'median [0-9.]*' $O/new_c3.txt) / barrier $(grep -o 'median [0-9.]*' $O/old_c3.txt)"
