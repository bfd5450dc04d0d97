# Round 4: phase cycles of the device WGL walk (LC_WGL_PROF variant, A/B
# diagnostics only) on C2, C5 and C4 at 2^16.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r4e
mkdir -p $O
export LINCHECK_LIB_OVERRIDE=jepsen-etcd-demo_amd/lincheck/liblincheck_wglprof.so
for c in C2 C5; do
  echo "== $c $(date +%T)"
  timeout -k 10 300 python -u tools/wgl_prof.py $c > $O/wglprof_$c.json 2> $O/wglprof_$c.err || { tail -5 $O/wglprof_$c.err; exit 1; }
  cat $O/wglprof_$c.json
done
echo "== C4 $(date +%T)"
timeout -k 10 300 python -u tools/wgl_prof.py C4 65536 > $O/wglprof_C4.json 2> $O/wglprof_C4.err || { tail -5 $O/wglprof_C4.err; exit 1; }
cat $O/wglprof_C4.json
echo ALL_OK
