"""SQ counters of one kernel from rocprofv3 --pmc passes (counter_collection
CSVs), per launch (median over dispatches), into a profiles/ JSON the bench
reads for roofline.issue: VALU / SALU instructions per launch, and the split
of the waves' cycles into issuing, issue-stalled and parked (MI355X_MICROARCH.md:
SQ_WAIT_ANY + SQ_WAIT_INST_ANY + SQ_ACTIVE_INST_ANY = SQ_WAVE_CYCLES, quad-cycles).
usage: sq_summary.py KERNEL_SUBSTR WORKLOAD BUDGET OUT CMD CSV..."""
import csv
import json
import statistics
import sys

kern, workload, budget, out, cmd = sys.argv[1:6]
vals, name = {}, None
for path in sys.argv[6:]:
    for r in csv.DictReader(open(path)):
        if kern in r["Kernel_Name"]:
            name = r["Kernel_Name"]
            vals.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
med = {k: statistics.median(v) for k, v in vals.items()}
import os
d = {"workload": workload, "kernel": name, "round": int(os.environ.get("LC_ROUND", "4")), "budget": int(budget),
     "command": cmd, "algorithm": os.environ.get("LC_ALGORITHM", "linear"),
     "dispatches": {k: len(v) for k, v in vals.items()}, "per_launch_median": med}
if "SQ_INSTS_VALU" in med:
    d["sq_insts_valu_per_launch"] = med["SQ_INSTS_VALU"]
if "SQ_INSTS_SALU" in med:
    d["sq_insts_salu_per_launch"] = med["SQ_INSTS_SALU"]
wc = med.get("SQ_WAVE_CYCLES")
if wc:
    for k in ("SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY"):
        if k in med:
            d[k.lower() + "_frac_of_wave_cycles"] = med[k] / wc
json.dump(d, open(out, "w"), indent=1)
print(json.dumps(d))
