# Round 6: k_wgl phase cycles (LC_WGL_PROF build) on C2, and C4 at 2^16 and 2^20.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6k; mkdir -p $O
export LINCHECK_LIB_OVERRIDE=$PWD/jepsen-etcd-demo_amd/lincheck/liblincheck_wglprof.so
timeout -k 10 200 python -u tools/wgl_prof.py C2 > $O/c2.json 2>$O/c2.err || { tail $O/c2.err; exit 1; }
timeout -k 10 200 python -u tools/wgl_prof.py C4 65536 > $O/c4_16.json 2>$O/c4_16.err || { tail $O/c4_16.err; exit 1; }
timeout -k 10 300 python -u tools/wgl_prof.py C4 1048576 > $O/c4_20.json 2>$O/c4_20.err || { tail $O/c4_20.err; exit 1; }
cat $O/c2.json $O/c4_16.json $O/c4_20.json
