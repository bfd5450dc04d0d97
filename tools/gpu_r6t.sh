# Round 6: phase stamps of the overlapped k_spec on C2 and C5 (raw, for the
# per-block critical path).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6t; mkdir -p $O
export LINCHECK_LIB_OVERRIDE=$PWD/jepsen-etcd-demo_amd/lincheck/liblincheck_specst.so
SPEC_CFG=C2 timeout -k 10 120 python -u tools/spec_stamps.py 1000 8 0 $O/st_c2.npz > $O/st_c2.txt 2>&1 || { tail $O/st_c2.txt; exit 1; }
SPEC_CFG=C5 timeout -k 10 120 python -u tools/spec_stamps.py 1000 8 0 $O/st_c5.npz > $O/st_c5.txt 2>&1 || { tail $O/st_c5.txt; exit 1; }
head -12 $O/st_c2.txt
