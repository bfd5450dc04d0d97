# Round 6: the GPU suite and bench lines on the current build, C5's kernel
# trace, the C5 phase stamps saved raw (per-XCD tail), and C4 :wgl at 2^24
# with the CPU restatement on all 256 keys.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
PARTS="tests c2 c5 c5jepsen" R=6e bash tools/gpu_evidence.sh || exit 1
O=gpurun_out/r6e
LINCHECK_LIB_OVERRIDE=$PWD/jepsen-etcd-demo_amd/lincheck/liblincheck_specst.so SPEC_CFG=C5 \
  timeout -k 10 120 python -u tools/spec_stamps.py 1000 8 0 $O/st_c5_8.npz > $O/st_c5_8.txt 2>&1 || { tail $O/st_c5_8.txt; exit 1; }
PARTS="c4wgl24" R=6e bash tools/gpu_evidence.sh || exit 1
