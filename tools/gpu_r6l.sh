# Round 6: k_wgl with the probe loads issued together -- the WGL tests,
# C4 :wgl at 2^16 and C2 :wgl lines, and the phase cycles (LC_WGL_PROF build).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6l; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_wgl.py tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 400 python -u bench.py --config C4 --budget 65536 --algorithm wgl --steps 3 --warmup 1 --no-resident > $O/c4wgl.json 2> $O/c4wgl.err || { tail $O/c4wgl.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/c4wgl.json').read().strip().splitlines()[-1]); print('C4 wgl 2^16', d['ms_per_step'], d['wgl']['ms_per_launch'], d['verdicts'], d['parity_vs_oracle'])"
timeout -k 10 400 python -u bench.py --config C2 --algorithm wgl --steps 10 --warmup 2 --no-resident --no-c3 > $O/c2wgl.json 2> $O/c2wgl.err || { tail $O/c2wgl.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/c2wgl.json').read().strip().splitlines()[-1]); print('C2 wgl', d['ms_per_step'], d['wgl']['ms_per_launch'], d['verdicts'], d['parity_vs_oracle'])"
export LINCHECK_LIB_OVERRIDE=$PWD/jepsen-etcd-demo_amd/lincheck/liblincheck_wglprof.so
timeout -k 10 200 python -u tools/wgl_prof.py C4 65536 > $O/c4_16.json 2>$O/c4_16.err || { tail $O/c4_16.err; exit 1; }
timeout -k 10 200 python -u tools/wgl_prof.py C2 > $O/c2.json 2>$O/c2.err || { tail $O/c2.err; exit 1; }
cat $O/c4_16.json $O/c2.json
