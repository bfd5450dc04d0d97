"""rocprofv3 --pmc passes of one kernel -> a profiles/ JSON that bench.py reads
for roofline.traffic (`bytes`) and roofline.issue (`sq`).

Only WHOLE launches are summarised.  A command can launch the same kernel at
several sizes -- a large shard's synchronous step searches 4 key chunks, one
launch each, beside the pipelined steps' whole-shard launches -- and counters
of a chunk divided by a whole launch's time and bytes are wrong by the chunk
factor.  So the dispatches kept are those whose grid
(rocprof's Grid_Size, work-items) equals the largest grid among the kernel's
dispatches in the pass; the JSON records that grid, the workgroup count, the
key count of the workload and how many dispatches were kept of how many, and
bench.py refuses a profile whose key count or launch shape differs from the
launch it divides by.

  bytes: FETCH_SIZE / WRITE_SIZE (KB per dispatch) corrected as
         MI355X_MICROARCH.md section HBM prescribes (FETCH_SIZE x 2 on gfx950,
         checked at 2-16 B/lane in profiles/r04_fetch_calib.json):
         bytes_per_launch = (2 x FETCH + WRITE) x 1024.
  sq:    SQ_* counters per launch (median over the kept dispatches): VALU /
         SALU instructions, and the waves' cycles split into issuing,
         issue-stalled and parked (SQ_WAIT_ANY + SQ_WAIT_INST_ANY +
         SQ_ACTIVE_INST_ANY = SQ_WAVE_CYCLES).

usage:
  profile_summary.py bytes --kernel SUBSTR --workload C3 --keys 12500 --budget B --round 5 \
      --out profiles/r05_c3s_pmc.json --cmd "..." FETCH_CSV WRITE_CSV
  profile_summary.py sq    --kernel SUBSTR ... --out profiles/r05_c3s_sq.json CSV [CSV ...]
"""

import argparse
import csv
import json
import os
import statistics
import sys


def dispatches(paths, kern):
    """{dispatch id: {"name", "grid", "wg", "counters": {name: value}}} of the
    kernel's dispatches in the counter_collection CSVs of one or more passes
    (a pass's dispatch ids are its own: keyed by (pass, id))."""
    out = {}
    for pi, path in enumerate(paths):
        for r in csv.DictReader(open(path)):
            if kern not in r["Kernel_Name"]:
                continue
            d = out.setdefault((pi, int(r["Dispatch_Id"])), {
                "name": r["Kernel_Name"], "grid": int(r["Grid_Size"]), "wg": int(r["Workgroup_Size"]),
                "counters": {}})
            d["counters"][r["Counter_Name"]] = d["counters"].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return out


def whole(ds):
    """The dispatches of the largest grid (whole launches), and a shape record."""
    if not ds:
        raise SystemExit("no dispatch of the kernel in the pass(es)")
    g = max(d["grid"] for d in ds.values())
    kept = {k: d for k, d in ds.items() if d["grid"] == g}
    wg = next(iter(kept.values()))["wg"]
    grids = sorted({d["grid"] for d in ds.values()})
    shape = {"grid_size": g, "workgroup_size": wg, "workgroups": g // max(wg, 1),
             "dispatches_kept": len(kept), "dispatches_total": len(ds), "other_grids": grids[:-1],
             "whole_launch": True}
    return kept, shape


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("mode", choices=("bytes", "sq", "trace"))
    ap.add_argument("--kernel", required=True)
    ap.add_argument("--workload", required=True)
    ap.add_argument("--keys", type=int, required=True, help="keys of the launch the bench divides by")
    ap.add_argument("--budget", type=int, required=True)
    ap.add_argument("--round", type=int, required=True)
    ap.add_argument("--algorithm", default="linear")
    ap.add_argument("--out", required=True)
    ap.add_argument("--cmd", default="")
    ap.add_argument("csvs", nargs="+")
    a = ap.parse_args()
    base = {"workload": a.workload, "keys": a.keys, "budget": a.budget, "round": a.round,
            "algorithm": a.algorithm, "command": a.cmd, "passes": a.csvs}
    if a.mode == "trace":
        # rocprofv3 --kernel-trace: the average duration of the kernel's whole
        # launches (the stats CSV averages every launch of the command,
        # chunk launches of a synchronous large-shard step included)
        rows = [r for r in csv.DictReader(open(a.csvs[0])) if a.kernel in r["Kernel_Name"]]
        if not rows:
            raise SystemExit("no dispatch of the kernel in the trace")
        gx = lambda r: int(r["Grid_Size_X"]) * int(r.get("Grid_Size_Y", 1) or 1) * int(r.get("Grid_Size_Z", 1) or 1)
        g = max(gx(r) for r in rows)
        kept = [r for r in rows if gx(r) == g]
        durs = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in kept]
        d = dict(base, kernel=kept[0]["Kernel_Name"], grid_size=g,
                 workgroup_size=int(kept[0]["Workgroup_Size_X"]),
                 workgroups=g // max(int(kept[0]["Workgroup_Size_X"]), 1), whole_launch=True,
                 dispatches_kept=len(kept), dispatches_total=len(rows),
                 avg_ms_whole_launch=statistics.mean(durs), min_ms=min(durs), max_ms=max(durs),
                 avg_ms_all_launches=statistics.mean((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
                                                     for r in rows))
    elif a.mode == "bytes":
        if len(a.csvs) != 2:
            raise SystemExit("bytes: FETCH_CSV WRITE_CSV")
        f, sf = whole(dispatches([a.csvs[0]], a.kernel))
        w, sw = whole(dispatches([a.csvs[1]], a.kernel))
        if sf["grid_size"] != sw["grid_size"]:
            raise SystemExit(f"FETCH and WRITE passes disagree on the whole launch: {sf} / {sw}")
        fk = statistics.median(d["counters"]["FETCH_SIZE"] for d in f.values())
        wk = statistics.median(d["counters"]["WRITE_SIZE"] for d in w.values())
        d = dict(base, kernel=next(iter(f.values()))["name"], **sf,
                 dispatches=[len(f), len(w)], fetch_size_kb_raw_median=fk, write_size_kb_raw_median=wk,
                 fetch_correction="x2 (MI355X_MICROARCH.md section HBM; validated on gfx950 at 2, 4, 8 and 16 "
                                  "B/lane: profiles/r04_fetch_calib.json)",
                 bytes_per_launch=int(round((2 * fk + wk) * 1024)))
    else:
        kept, shape = whole(dispatches(a.csvs, a.kernel))
        # each pass has its own whole launches: a counter's median over the
        # kept dispatches of the pass(es) that collected it
        vals = {}
        for dd in kept.values():
            for k, v in dd["counters"].items():
                vals.setdefault(k, []).append(v)
        med = {k: statistics.median(v) for k, v in vals.items()}
        d = dict(base, kernel=next(iter(kept.values()))["name"], **shape,
                 dispatches={k: len(v) for k, v in vals.items()}, per_launch_median=med)
        if "SQ_INSTS_VALU" in med:
            d["sq_insts_valu_per_launch"] = med["SQ_INSTS_VALU"]
        if "SQ_INSTS_SALU" in med:
            d["sq_insts_salu_per_launch"] = med["SQ_INSTS_SALU"]
        if "SQ_WAVES" in med:
            d["sq_waves_per_launch"] = med["SQ_WAVES"]
        wc = med.get("SQ_WAVE_CYCLES")
        if wc:
            for k in ("SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY"):
                if k in med:
                    d[k.lower() + "_frac_of_wave_cycles"] = med[k] / wc
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    json.dump(d, open(a.out, "w"), indent=1)
    print(json.dumps({k: d[k] for k in ("kernel", "grid_size", "dispatches_kept", "dispatches_total")}))
    return 0


if __name__ == "__main__":
    sys.exit(main())
