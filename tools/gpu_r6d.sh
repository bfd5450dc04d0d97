set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6d; mkdir -p $O
export LINCHECK_LIB_OVERRIDE=$PWD/jepsen-etcd-demo_amd/lincheck/liblincheck_specst.so
SPEC_CFG=C5 timeout -k 10 120 python -u tools/spec_stamps.py 1000 8 > $O/st_c5_8.txt 2>&1 || { tail $O/st_c5_8.txt; exit 1; }
SPEC_CFG=C5 timeout -k 10 120 python -u tools/spec_stamps.py 1000 4 > $O/st_c5_4.txt 2>&1 || { tail $O/st_c5_4.txt; exit 1; }
SPEC_CFG=C2 timeout -k 10 120 python -u tools/spec_stamps.py 1000 8 > $O/st_c2_8.txt 2>&1 || { tail $O/st_c2_8.txt; exit 1; }
tail -8 $O/st_c5_8.txt; tail -8 $O/st_c5_4.txt; tail -8 $O/st_c2_8.txt
