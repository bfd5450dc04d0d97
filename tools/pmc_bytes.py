"""Per-launch HBM traffic of one kernel from two rocprofv3 --pmc passes
(FETCH_SIZE, WRITE_SIZE; KB per dispatch), corrected as MI355X_MICROARCH.md
section HBM prescribes (FETCH_SIZE x 2 on gfx950).  Writes a profiles/ JSON.
usage: pmc_bytes.py KERNEL_SUBSTR FETCH_CSV WRITE_CSV WORKLOAD BUDGET OUT CMD [ROUND]"""
import csv, json, statistics, sys

kern, fcsv, wcsv, workload, budget, out, cmd = sys.argv[1:8]
rnd = int(sys.argv[8]) if len(sys.argv) > 8 else 4


def per_dispatch(path, counter):
    vals, name = [], None
    for r in csv.DictReader(open(path)):
        if kern in r["Kernel_Name"] and r["Counter_Name"] == counter:
            vals.append(float(r["Counter_Value"]))
            name = r["Kernel_Name"]
    return vals, name


f, name = per_dispatch(fcsv, "FETCH_SIZE")
w, _ = per_dispatch(wcsv, "WRITE_SIZE")
fk, wk = statistics.median(f), statistics.median(w)
import os
d = {"workload": workload, "kernel": name, "round": rnd, "dispatches": [len(f), len(w)],
     "algorithm": os.environ.get("LC_ALGORITHM", "linear"),
     "fetch_size_kb_raw_median": fk, "write_size_kb_raw_median": wk,
     "fetch_correction": "x2 (MI355X_MICROARCH.md section HBM; validated on gfx950 at 2, 4, 8 and 16 B/lane: "
                         "profiles/r04_fetch_calib.json)",
     "bytes_per_launch": int(round((2 * fk + wk) * 1024)), "command": cmd,
     "passes": [fcsv, wcsv], "budget": int(budget)}
json.dump(d, open(out, "w"), indent=1)
print(json.dumps(d))
