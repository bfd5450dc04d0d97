"""can the device decide BASELINE config C4 (256 keys x 5,000
ops, concurrency 30, 2 % crashed write/cas) at a larger search budget?

For each algorithm (:linear = the layered HBM tier, :wgl = knossos.wgl's walk)
and budget, one full-C4 lc_check_batch on the device: verdict counts, the
event each :unknown key gave up at (:linear: the `:ok` whose set passed the
budget -> "events reached"), time per launch, WGL steps and cache sizes; and
the C restatements (oracle/linear_ref.c, oracle/wgl_ref.c) on the batch's
first `--sample` keys at the same budget, records compared.  Test
infrastructure (under tests/ because it runs the oracle as the checker); the
product path it measures is liblincheck.so.

    python tests/tools/c4_budget_sweep.py --budgets 16,18,20,22 --algos linear,wgl \
        --sample 16 --out gpurun_out/c4sweep.json

Writes the JSON after every point (a long sweep that is cut off keeps what it
measured) and prints one progress line per point.
"""

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (os.path.join(ROOT, "jepsen-etcd-demo_amd"), os.path.join(ROOT, "oracle")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402

ALGOS = {"linear": 0, "wgl": 1}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--budgets", default="16,18,20,22", help="log2 budgets")
    ap.add_argument("--algos", default="linear,wgl")
    ap.add_argument("--sample", type=int, default=16, help="keys checked by the C oracle at each point (0: none)")
    ap.add_argument("--oracle-max-log2", type=int, default=22, help="skip the oracle sample above this budget")
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--keys", type=int, default=256)
    ap.add_argument("--out", default="gpurun_out/c4sweep.json")
    args = ap.parse_args()

    import cref
    from lincheck import history as H
    from lincheck.checker import Device, Packed

    t = time.perf_counter()
    hist = H.synth(n_keys=args.keys, ops_per_key=5000, concurrency=30, info_rate=0.02, seed=4)
    packed = Packed(hist)
    K = packed.n_keys
    n_ev = np.diff(packed.ev_off.astype(np.int64))
    print(f"C4 {K} keys, {int(n_ev.sum())} events, packed in {time.perf_counter() - t:.1f} s", flush=True)
    sample = min(args.sample, K)
    sub = H.synth(n_keys=sample, ops_per_key=5000, concurrency=30, info_rate=0.02, seed=4) if sample else None
    out = {"workload": "C4: 256 keys x 5,000 ops, concurrency 30, 2% crashed write/cas, seed 4",
           "keys": K, "events": int(n_ev.sum()), "oracle_sample_keys": sample, "points": []}

    def dump():
        os.makedirs(os.path.dirname(os.path.abspath(args.out)), exist_ok=True)
        with open(args.out, "w") as f:
            json.dump(out, f, indent=1)

    for algo in args.algos.split(","):
        for lb in (int(x) for x in args.budgets.split(",")):
            budget = 1 << lb
            pt = {"algorithm": algo, "budget": budget, "log2_budget": lb}
            t = time.perf_counter()
            try:
                dev = Device(0, budget=budget, algorithm=ALGOS[algo])
                res = dev.check(packed)
            except Exception as e:  # noqa: BLE001 -- record and go on (e.g. workspace too large)
                pt["error"] = repr(e)
                out["points"].append(pt)
                dump()
                print(json.dumps(pt), flush=True)
                continue
            wall = time.perf_counter() - t
            v = res.valid.astype(np.int64)
            unk = v == -1
            fe = res.fail_event.astype(np.int64)
            reached = np.where(unk & (fe >= 0), fe / np.maximum(n_ev, 1), np.nan)
            st = res.stats
            pt.update({
                "valid": int((v == 1).sum()), "invalid": int((v == 0).sum()), "unknown": int(unk.sum()),
                "decided": int((v != -1).sum()),
                "causes": {str(c): int((res.cause == c).sum()) for c in np.unique(res.cause)},
                "wall_s": round(wall, 3), "kernel_ms": st["kernel_ms"], "tier3_ms": st["tier3_ms"],
                "wgl_ms": st["wgl_ms"], "wgl_steps": int(st["wgl_steps"]), "wgl_spilled": int(st["wgl_spilled"]),
                "peak_median": int(np.median(res.peak)), "peak_max": int(res.peak.max()),
            })
            if algo == "linear" and unk.any():
                r = reached[~np.isnan(reached)]
                if r.size:
                    pt["unknown_event_reached_frac"] = {"min": float(r.min()), "median": float(np.median(r)),
                                                        "max": float(r.max())}
                    pt["unknown_fail_event_median"] = int(np.median(fe[unk & (fe >= 0)]))
            if sample and lb <= args.oracle_max_log2:
                to = time.perf_counter()
                if algo == "linear":
                    _, orc = cref.check_history(sub.as_c(), budget=budget, threads=args.threads)
                    same = (np.array_equal(orc["valid"], res.valid[:sample])
                            and np.array_equal(orc["fail_event"], res.fail_event[:sample])
                            and np.array_equal(orc["cause"], res.cause[:sample]))
                else:
                    _, orc, _, _ = cref.check_history_wgl(sub.as_c(), budget=budget, threads=args.threads)
                    same = (np.array_equal(orc["valid"], res.valid[:sample])
                            and np.array_equal(orc["fail_event"], res.fail_event[:sample])
                            and np.array_equal(orc["cause"], res.cause[:sample])
                            and np.array_equal(orc["peak"], res.peak[:sample]))
                pt["oracle"] = {"keys": sample, "same_records": bool(same), "cpu_s": round(time.perf_counter() - to, 2),
                                "threads": args.threads, "decided": int((orc["valid"] != -1).sum())}
            del dev
            out["points"].append(pt)
            dump()
            print(json.dumps(pt), flush=True)
    dump()


if __name__ == "__main__":
    main()
