# Timeline of C2 D-1 steps: kernels and memory copies (rocprofv3 traces, no counters).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/tl
mkdir -p $O
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace -d $O/t -o t --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu --no-resident --no-probes > $O/t.log 2>&1 || { tail -20 $O/t.log; exit 1; }
python3 - <<'PY'
import csv, glob
rows=[]
for f in glob.glob("gpurun_out/tl/t/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)): rows.append((int(r['Start_Timestamp']), int(r['End_Timestamp']), 'K '+r['Kernel_Name'][:40]))
for f in glob.glob("gpurun_out/tl/t/**/*memory_copy_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)): rows.append((int(r['Start_Timestamp']), int(r['End_Timestamp']), 'M '+r.get('Direction','?')+' '+r.get('Size', r.get('Bytes','?'))))
rows.sort()
ks=[i for i,r in enumerate(rows) if 'k_spec<' in r[2]]
a,b=ks[-4],ks[-2]
t0=rows[a][0]
for s,e,n in rows[a-6:b+1]:
    print("%9.1f %8.1f  %s" % ((s-t0)/1000,(e-s)/1000,n))
PY
echo ALL_OK
