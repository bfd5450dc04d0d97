# SQ counters of k_spec<4> on the C2 bench step (two --pmc passes).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/specsq
mkdir -p $O
B="python3 bench.py --steps 5 --warmup 1 --no-cpu --no-resident --no-probes"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU -d $O/p1 -o p1 --output-format csv -- $B > $O/p1.log 2>&1 || { tail -5 $O/p1.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_SMEM -d $O/p2 -o p2 --output-format csv -- $B > $O/p2.log 2>&1 || { tail -5 $O/p2.log; exit 1; }
python3 - <<'PY'
import csv, glob, collections
for p in ("p1", "p2"):
    f = glob.glob(f"gpurun_out/specsq/{p}/**/*counter_collection.csv", recursive=True)[0]
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "k_spec<" not in k and "k_widen" not in k: continue
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, d in acc.items():
        print(p, k[:40], {c: sorted(v)[len(v)//2] for c, v in d.items()})
PY
echo ALL_OK
