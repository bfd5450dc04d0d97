# Register-tier A/B: tools/spec_ab.py on C2 and C5 (settings as arguments), then the spec tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/specab
mkdir -p $O
S=${SETTINGS:-"default path_flags=0x100 path_flags=0x500 path_flags=0x700 path_flags=0x400"}
timeout -k 10 300 python -u tools/spec_ab.py C2 1000 1000 $S > $O/ab_c2.txt 2>&1 || { tail -5 $O/ab_c2.txt; exit 1; }
cat $O/ab_c2.txt
timeout -k 10 300 python -u tools/spec_ab.py C5 1000 1000 $S > $O/ab_c5.txt 2>&1 || { tail -5 $O/ab_c5.txt; exit 1; }
cat $O/ab_c5.txt
if [ -z "$NOTEST" ]; then
timeout -k 10 600 python -u -m pytest tests/test_gpu_spec.py tests/test_gpu_events16.py -v -x --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { grep -E "FAILED|Error" $O/tests.log | head; tail -3 $O/tests.log; exit 1; }
tail -1 $O/tests.log
fi
echo ALL_OK
