"""Benchmark: history ops linearizability-checked per second (BASELINE.json metric).

`value` is SURVEY.md 8(d) D-1's rate: timed end to end from each rank's
shard of packed struct-of-arrays in host memory to the node's verdict
records -- lc_check_node_async, two steps in flight (H2D -> search -> verdict
records -> all-gather of every rank's records over RCCL -> records in
page-locked host memory; each step's upload overlaps the search before it),
K steps between barriers, the slowest rank's time.  Reported beside it:
`resident` (the same step with the shard already resident in HBM when the
timed region starts: lc_check_node_device, asynchronous, HIP-event span per
launch -- the kernel-side rate, never `value`), `d1_pipelined` (the same
numbers as `value`, kept under their round-5 name) and `d1_sync`
(lc_check_node, one step at a time; the roofline's per-launch times of the
set tiers come from those synchronous steps).

Workloads (BASELINE.json configs; synthetic, liblincheck's seeded generator):
  N = 1 (default): C2, 1,000 keys x 1,000 client ops, concurrency 10,
        cas-register over values 0..4 (etcdemo.clj:67-69), seed 2 -- the
        `value`.  The same run then checks C3's whole key space on this one
        GPU (`c3_strong`: the N = 1 point of the 2/4/8-GPU curve, measured by
        the same command; --no-c3 skips it).
  N > 1 (default): C3, 100,000 keys x 2,000 ops in total, concurrency 10,
        contiguous key shards, one per rank (strong scaling).
  --config C1|C4|C5 select the others (C1: history.edn -> result map, the
  demo's check phase end to end).
Every line carries the host marshalling cost beside the step: `pack_ms` /
`pack_ops_per_s` time lc_pack alone (history -> packed SoA)
on the history the step consumes; `synth_s` is the generator's time.

Also reported (one JSON line on rank 0):
  roofline      the dominant kernel's algorithmic HBM bytes per launch over
                its average HIP-event launch time in the timed steps
                (DESIGN.md section 5), MI355X peak 8 TB/s; traffic from
                profiles/*pmc*.json when committed for this workload.
  cpu_baseline  the C restatement of knossos.linear (oracle/linear_ref.c,
                kind "port") on this host's cores and on one core, on a
                bounded sample of the same workload (rank 0, N = 1); `wgl`
                beside it: the C restatement of knossos.wgl
                (oracle/wgl_ref.c) on the same cores and sample.

--algorithm wgl|competition runs the step with lc_opts.algorithm
LC_ALGO_WGL (knossos.wgl's walk on the device: device_wgl.hip) or
LC_ALGO_COMPETITION (:linear, then WGL for its budget keys); the line then
names k_wgl as the dominant kernel where it is.  --jepsen times the drop-in's
real call instead: independent/checker(compose {:linear linearizable,
:timeline}) from the packed history to Knossos-shaped result maps (exact-set
search with final configs, counterexamples for the invalid keys), with the
pack / search / shaping split reported.
"""

import argparse
import glob
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for p in (os.path.join(ROOT, "jepsen-etcd-demo_amd"), os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
# profiles/*.json summaries (rocprofv3 --pmc / SQ) are used for `traffic` /
# `issue` only when they were taken of this round's build
PROFILE_ROUND = 6
ALGORITHMS = {"linear": 0, "wgl": 1, "competition": 2}
SHADER_CLOCK_HZ = 2.4e9  # MI355X peak engine clock
METRIC = "history ops linearizability-checked/sec (whole node)"

CONFIGS = {
    "C2": dict(keys=1000, ops=1000, concurrency=10, info_rate=0.0, anomaly_rate=0.0, seed=2,
               desc="C2: 1,000 keys x 1,000 ops per GPU, concurrency 10, cas-register values 0..4, all linearizable"),
    "C3": dict(keys=100_000, ops=2000, concurrency=10, info_rate=0.0, anomaly_rate=0.0, seed=3, strong=True,
               desc="C3: 100,000 keys x 2,000 ops in total, concurrency 10, keys sharded over the GPUs"),
    "C4": dict(keys=256, ops=5000, concurrency=30, info_rate=0.02, anomaly_rate=0.0, seed=4,
               desc="C4: 256 keys x 5,000 ops, concurrency 30, 2% crashed write/cas"),
    "C1": dict(keys=6, ops=100, concurrency=10, info_rate=0.0, anomaly_rate=0.0, seed=1,
               desc="C1: demo re-check, history.edn of 6 keys x 100 ops, 10 clients, nemesis :info ops "
                    "(the stored run is absent: synthetic file of the demo's shape)"),
    "C5": dict(keys=1000, ops=1000, concurrency=10, info_rate=0.0, anomaly_rate=0.05, seed=5,
               desc="C5: C2 shape with stale reads / lost cas in 5% of keys"),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default=None, choices=sorted(CONFIGS),
                    help="default: C2 at one GPU, C3 (strong scaling) at more")
    ap.add_argument("--budget", type=int, default=1 << 20)
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline")
    ap.add_argument("--cpu-full", action="store_true",
                    help="time the CPU :wgl restatement on the whole batch, not a bounded sample")
    ap.add_argument("--no-resident", action="store_true", help="skip the resident-shard steps")
    ap.add_argument("--d1-sync", action="store_true",
                    help="time the synchronous lc_check_node step instead of the pipelined one")
    ap.add_argument("--no-probes", action="store_true", help="skip the probe-counting pass")
    ap.add_argument("--no-c3", action="store_true", help="N = 1: skip the C3-on-one-GPU block (c3_strong)")
    ap.add_argument("--c3-steps", type=int, default=10, help="timed pipelined steps of the c3_strong block")
    ap.add_argument("--algorithm", default="linear", choices=sorted(ALGORITHMS),
                    help="lc_opts.algorithm of the step (jepsen.checker/linearizable's :algorithm)")
    ap.add_argument("--jepsen", action="store_true",
                    help="time independent/checker(compose{linearizable, timeline}) -> result maps")
    ap.add_argument("--keys", type=int, default=0, help="override keys (exploration only)")
    ap.add_argument("--ops", type=int, default=0, help="override ops per key (exploration only)")
    ap.add_argument("--path-flags", type=lambda x: int(x, 0), default=0,
                    help="lc_opts.path_flags (LC_PATH_*) of the step: pinned path choices for A/B runs only")
    return ap.parse_args()


def host_cores():
    """(nproc, CPUs this process may run on, CPUs its cgroup quota allows)."""
    nproc = os.cpu_count() or 1
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = nproc
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, math.ceil(int(q) / int(per)))
    except (OSError, ValueError):
        pass
    return nproc, aff, quota


def bench_c1(args):
    """C1 (BASELINE.json configs[0]): the demo's check phase end to end, as
    etcdemo.clj:115-119 runs it -- history.edn on disk -> lc_edn_read ->
    independent/checker over compose {:linear linearizable, :timeline} ->
    the result map.  A step is that whole call."""
    import tempfile

    import numpy as np

    from lincheck import checker as CK
    from lincheck import history as H
    from lincheck import independent as IND
    from lincheck import model as M

    hist = H.synth(n_keys=6, ops_per_key=100, concurrency=10, interleave=True, nemesis_period=5.0, seed=1)
    path = os.path.join(tempfile.mkdtemp(), "history.edn")
    H.write_edn(path, hist)
    lin = CK.linearizable({"model": M.cas_register(), "algorithm": "linear", "max-configs": args.budget})
    chk = IND.checker(CK.compose({"linear": lin, "timeline": CK.unbridled_optimism()}))

    def step():
        return chk.check({}, H.read_edn(path), {})

    for _ in range(args.warmup):
        step()
    ts = []
    for _ in range(args.steps):
        t = time.perf_counter()
        out = step()
        ts.append(time.perf_counter() - t)
    elapsed = float(np.sum(ts))
    n_ops = 6 * 100
    cpu = parity = None
    if not args.no_cpu:
        import cref
        tc = time.perf_counter()
        reps = 0
        while time.perf_counter() - tc < 2.0:
            keys, orc = cref.check_history(H.read_edn(path).as_c(), budget=args.budget, threads=1)
            reps += 1
        tcpu = (time.perf_counter() - tc) / reps
        cpu = {"value": n_ops / tcpu, "unit": "ops/s", "cores": 1, "kind": "port",
               "sample": f"same history.edn read + oracle/linear_ref.c, 1 thread, {reps} reps of {tcpu * 1e3:.2f} ms"}
        fails = sorted(k for k, r in zip(keys, orc) if r["valid"] == 0)
        parity = bool(sorted(out["failures"]) == fails and out["valid?"] == (not fails))
    line = {
        "metric": METRIC, "value": n_ops * args.steps / elapsed, "unit": "ops/s", "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u32", "data": "synthetic",
        "config": {"workload": CONFIGS["C1"]["desc"], "keys_per_gpu": 6, "ops_per_key": 100, "concurrency": 10,
                   "budget": args.budget, "parallelism": "1 GPU (latency case)"},
        "roofline": None,
        "cpu_baseline": cpu,
        "step": "lc_edn_read + independent/checker(compose(linearizable, timeline)) -> result map",
        "valid?": out["valid?"], "failures": out["failures"], "parity_vs_oracle": parity,
    }
    print(json.dumps(line, default=str), flush=True)


def bench_jepsen(args):
    """The drop-in's real call (etcdemo.clj:115-119): independent/checker over
    compose {:linear (linearizable {:model cas-register}) :timeline} from the
    history to Knossos-shaped result maps -- lc_pack, lc_check_batch with
    final configs (the exact-set segmented search), then every key's result
    map and the counterexamples (lc_report, :final-paths) of the invalid
    ones.  A step is that whole call; the split into packing, search and
    shaping is reported beside it (Linearizable.last_timing)."""
    import numpy as np
    import torch

    from lincheck import checker as CK
    from lincheck import history as H
    from lincheck import independent as IND
    from lincheck import model as M

    if args.config is None:
        args.config = "C5"
    cfg = dict(CONFIGS[args.config])
    if args.keys or args.ops:
        cfg["keys"] = args.keys or cfg["keys"]
        cfg["ops"] = args.ops or cfg["ops"]
    K, ops = cfg["keys"], cfg["ops"]
    hist = H.synth(n_keys=K, ops_per_key=ops, concurrency=cfg["concurrency"], info_rate=cfg["info_rate"],
                   anomaly_rate=cfg["anomaly_rate"], seed=cfg["seed"])
    lin = CK.linearizable({"model": M.cas_register(), "algorithm": args.algorithm, "max-configs": args.budget})
    chk = IND.checker(CK.compose({"linear": lin, "timeline": CK.unbridled_optimism()}))
    for _ in range(args.warmup):
        out = chk.check({}, hist, {})
    torch.cuda.synchronize()
    ts, parts = [], []
    for _ in range(args.steps):
        t = time.perf_counter()
        out = chk.check({}, hist, {})
        ts.append(time.perf_counter() - t)
        parts.append(lin.last_timing)
    torch.cuda.synchronize()
    elapsed = float(np.sum(ts))
    split = {k: float(np.mean([p[k] for p in parts])) for k in parts[0]}
    res = out["results"]
    n_valid = sum(r["valid?"] is True for r in res.values())
    n_bad = sum(r["valid?"] is False for r in res.values())
    parity = None
    if not args.no_cpu:
        # each key against the oracle of the analysis that answered it
        # (:analyzer -- competition answers :linear's budget keys with WGL)
        import cref
        keys, orc = cref.check_history(hist.as_c(), budget=args.budget, threads=16)
        worc = None
        if args.algorithm != "linear":
            _, worc, _, _ = cref.check_history_wgl(hist.as_c(), budget=args.budget, threads=16)
        fails = []
        for i, k in enumerate(keys):
            anl = res[int(k)]["linear"].get("analyzer", "linear") if "linear" in res[int(k)] else "linear"
            o = worc if anl == "wgl" else orc
            if o[i]["valid"] == 0:
                fails.append(int(k))
        parity = bool(sorted(out["failures"]) == sorted(fails))
    line = {
        "metric": METRIC, "value": (n_valid + n_bad) * ops * args.steps / elapsed, "unit": "ops/s", "n_gpus": 1,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u32", "data": "synthetic",
        "config": {"workload": cfg["desc"], "keys": K, "ops_per_key": ops, "concurrency": cfg["concurrency"],
                   "budget": args.budget, "algorithm": args.algorithm, "parallelism": "1 GPU"},
        "step": "independent/checker(compose {:linear linearizable, :timeline}) on the packed history -> "
                "result maps (lc_pack, lc_check_batch with final configs, lc_report for invalid keys)",
        "split_ms": split,
        "search_stats": {k: out["stats"].get(k) for k in ("kernel_ms", "tier0_ms", "t0_path", "wgl_ms", "wgl_keys")},
        "verdicts": {"valid": n_valid, "invalid": n_bad, "unknown": len(res) - n_valid - n_bad},
        "failures_equal_oracle": parity,
        "roofline": None, "cpu_baseline": None,
    }
    print(json.dumps(line, default=str), flush=True)


def cpu_linear(args, K, hist, ops, threads, first_keys, v_host, fe_host, nproc, aff, quota):
    """oracle/linear_ref.c on all usable cores, then one core (cpu_baseline's
    :linear part)."""
    import numpy as np

    import cref
    kp = min(K, threads)
    tc = time.perf_counter()
    keys, orc = cref.check_history(first_keys(kp).as_c(), budget=args.budget, threads=threads)
    tcpu = time.perf_counter() - tc
    ks = kp
    if kp < K:
        ks = K if tcpu * K / kp <= 12.0 else min(K, max(kp, int(kp * 12.0 / max(tcpu, 1e-6)) // kp * kp))
        if ks > kp:
            tc = time.perf_counter()
            keys, orc = cref.check_history(first_keys(ks).as_c(), budget=args.budget, threads=threads)
            tcpu = time.perf_counter() - tc
    # a whole batch that finishes in well under a second is checked again
    # until ~10 s of CPU work have been timed (the rate is their mean)
    reps = 1
    if ks == K and tcpu < 0.6:
        reps = min(20, int(math.ceil(0.6 / max(tcpu, 1e-6))))
        tc = time.perf_counter()
        for _ in range(reps):
            keys, orc = cref.check_history(hist.as_c(), budget=args.budget, threads=threads)
        tcpu = (time.perf_counter() - tc) / reps
    # one thread: as many of the first keys as ~6 s allow
    per_key_1 = tcpu * threads / ks
    k1 = max(1, min(ks, int(6.0 / max(per_key_1, 1e-6))))
    t1 = time.perf_counter()
    cref.check_history(first_keys(k1).as_c(), budget=args.budget, threads=1)
    t1 = time.perf_counter() - t1
    what = (f"full {args.config} batch ({K} keys x {ops} ops)" if ks == K
            else f"first {ks} of the {K} keys of the {args.config} batch ({ops} ops each)")
    cpu = {"value": ks * ops / tcpu, "unit": "ops/s", "cores": threads, "kind": "port",
           "sample": f"{what}, oracle/linear_ref.c, {threads} threads, "
                     + (f"{reps} runs of {tcpu:.3f} s" if reps > 1 else f"{tcpu:.2f} s"),
           "host": {"nproc": nproc, "affinity": aff, "cgroup_cpu_quota": quota},
           "one_thread": {"value": k1 * ops / t1, "cores": 1,
                          "sample": f"first {k1} keys of the batch, 1 thread, {t1:.2f} s"}}
    if args.algorithm == "linear":
        parity = bool(np.array_equal(orc["valid"], v_host[:ks]) and np.array_equal(orc["fail_event"], fe_host[:ks]))
    else:
        parity = None
    if ks < K:
        cpu["parity_sample_keys"] = ks
    return cpu, parity


def cpu_baseline(args, cfg, K, key0, hist, ops, v_host, fe_host, nproc, aff, quota):
    """oracle/linear_ref.c with a pthread pool over keys (independent/
    checker's pmap) on this host: all usable cores, then one core, each on a
    bounded sample of the same batch (~10-20 s of CPU work in all)."""
    import numpy as np

    import cref
    from lincheck import history as H
    threads = max(1, min(aff, quota or aff))

    def first_keys(k):  # the batch's first k keys (per-key seeded generator)
        if k == K:
            return hist
        return H.synth(n_keys=k, ops_per_key=ops, concurrency=cfg["concurrency"], info_rate=cfg["info_rate"],
                       anomaly_rate=cfg["anomaly_rate"], seed=cfg["seed"], key_base=key0)

    cpu, parity = None, None
    # :linear at a large budget on C4-shaped keys takes minutes per key sample
    # (54 s for 16 keys at 2^22, profiles/r05_c4_budget_sweep.json): a --algorithm
    # wgl line at such a budget times the restatement of knossos.wgl alone
    if not (args.algorithm == "wgl" and args.budget > (1 << 20)):
        cpu, parity = cpu_linear(args, K, hist, ops, threads, first_keys, v_host, fe_host, nproc, aff, quota)
    else:
        cpu = {"linear": "not timed: the budget is beyond a bounded sample of :linear on this workload",
               "cores": threads, "host": {"nproc": nproc, "affinity": aff, "cgroup_cpu_quota": quota}}
    # knossos.wgl's search (the other analysis jepsen.checker/linearizable
    # offers, north_star's "CPU :linear/:wgl"): oracle/wgl_ref.c on the same
    # cores, on as many of the batch's first keys as ~8 s allow
    kw = K if args.cpu_full else min(K, threads)
    tw = time.perf_counter()
    _, worc, _, _ = cref.check_history_wgl(first_keys(kw).as_c(), budget=args.budget, threads=threads)
    twc = time.perf_counter() - tw
    if kw < K:
        kw2 = K if twc * K / kw <= 8.0 else min(K, max(kw, int(kw * 8.0 / max(twc, 1e-6)) // kw * kw))
        if kw2 > kw:
            kw = kw2
            tw = time.perf_counter()
            _, worc, _, _ = cref.check_history_wgl(first_keys(kw).as_c(), budget=args.budget, threads=threads)
            twc = time.perf_counter() - tw
    wreps = 1
    if kw == K and twc < 0.6:
        wreps = min(20, int(math.ceil(0.6 / max(twc, 1e-6))))
        tw = time.perf_counter()
        for _ in range(wreps):
            _, worc, _, _ = cref.check_history_wgl(hist.as_c(), budget=args.budget, threads=threads)
        twc = (time.perf_counter() - tw) / wreps
    wwhat = (f"full {args.config} batch" if kw == K else f"first {kw} of the {K} keys of the {args.config} batch")
    cpu["wgl"] = {"value": kw * ops / twc, "unit": "ops/s", "cores": threads, "kind": "port",
                  "sample": f"{wwhat}, oracle/wgl_ref.c (knossos.wgl), {threads} threads, "
                            + (f"{wreps} runs of {twc:.3f} s" if wreps > 1 else f"{twc:.2f} s"),
                  "keys_decided": int((worc["valid"] != -1).sum()), "keys": kw}
    if args.algorithm == "wgl":
        parity = bool(np.array_equal(worc["valid"], v_host[:kw]) and np.array_equal(worc["fail_event"], fe_host[:kw]))
    if "value" not in cpu:  # (the --algorithm wgl line at a large budget: knossos.wgl's restatement)
        cpu.update({k: cpu["wgl"][k] for k in ("value", "unit", "kind", "sample")})
    return cpu, parity


def profile_mismatch(d, K, kname):
    """Why a profiles/ summary does not describe the launch the line divides
    by (None when it does): its key count, and whole launches only."""
    if d.get("keys") != K:
        return f"profile of {d.get('keys')} keys, launch of {K}"
    if not d.get("whole_launch") or not d.get("grid_size"):
        return "no whole-launch grid recorded (a median over dispatches of mixed size)"
    if ("k_spec" in kname or "k_search_lattice" in kname) and d.get("workgroups", 0) < K:
        # the register tier runs one workgroup per key (plus validation blocks)
        return f"{d.get('workgroups')} workgroups < {K} keys: a chunk launch"
    return None


def probe_rates(probes, probes_t3, avg_t0, avg_t3, d1_t3, wgl):
    """Probes per second of each tier's launch (None where not measured)."""
    out = {}
    if probes is not None and avg_t0 > 0:
        t0p = probes - (probes_t3 or 0)
        out["t0"] = t0p / (avg_t0 * 1e-3) if t0p > 0 else None
    if probes_t3 and avg_t3 > 0:
        out["t3"] = probes_t3 / (avg_t3 * 1e-3)
    if wgl and wgl.get("probes") and wgl.get("ms_per_launch"):
        out["wgl"] = wgl["probes"] / (wgl["ms_per_launch"] * 1e-3)
    return out or None


def bench_c3_strong(args, local):
    """C3's whole key space (100,000 keys x 2,000 ops) on this one GPU: the
    N = 1 point of the strong-scaling curve that `bench.py --gpus N` measures
    with the same step (lc_check_node_async, pipelined), so the driver's
    2/4/8-GPU runs have a same-workload base from the default command.  Also
    the host side at C3 scale: generator and lc_pack times.
    Verdicts are property-checked (C3 has no anomalies: every key valid)."""
    import numpy as np
    import torch

    from lincheck import _native as NN
    from lincheck import history as H
    from lincheck import parallel as P
    from lincheck.checker import Device, Packed, PinnedRecords
    cfg = CONFIGS["C3"]
    t = time.perf_counter()
    hist = H.synth(n_keys=cfg["keys"], ops_per_key=cfg["ops"], concurrency=cfg["concurrency"], seed=cfg["seed"])
    synth_s = time.perf_counter() - t
    t = time.perf_counter()
    packed = Packed(hist)
    pack_s = time.perf_counter() - t
    K, n_ev = packed.n_keys, int(packed.ev_off[-1])
    print(f"[c3_strong] {K} keys synthesised in {synth_s:.1f} s, packed in {pack_s:.2f} s", file=sys.stderr, flush=True)
    dev = Device(local, budget=args.budget)
    buf = PinnedRecords(K)
    dev.check_node_async(packed, K, buf)  # warmup (allocations, first upload)
    dev.wait()
    torch.cuda.synchronize()
    steps = max(1, args.c3_steps)
    t = time.perf_counter()
    for _ in range(steps):
        dev.check_node_async(packed, K, buf)
    dev.wait()
    torch.cuda.synchronize()
    el = time.perf_counter() - t
    v, c, fe = P.unpack_records(np.asarray(buf)[:K].astype(np.int64))
    # the same steps with the key space resident in HBM (reported beside
    # the D-1 rate, never as it)
    db = dev.upload(packed)
    db.check_node(K, asynchronous=True)
    dev.wait()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(steps):
        db.check_node(K, asynchronous=True)
    dev.wait()
    torch.cuda.synchronize()
    el_r = time.perf_counter() - t
    same_r = bool(np.array_equal(dev.node_records(K), np.asarray(buf)[:K]))
    del db
    _, st = dev.check_node(packed, K)  # one synchronous step: the register tier's launch time
    ops_total = cfg["keys"] * cfg["ops"]
    ewb = int(st.ev_word_bytes) or 4
    alg = ewb * n_ev + 8 * (K + 1) + 4 * K + 4 * int(packed.view.n_trans) + 8 * K
    # the same history packed again, as a checker that packs a history per
    # check does after its first: the library's host blocks (page-locked
    # output, staging) come from its caches instead of fresh pages
    del packed
    t = time.perf_counter()
    packed = Packed(hist)
    pack_warm_s = time.perf_counter() - t
    out = {"workload": cfg["desc"] + " -- all on one GPU", "keys": K, "ops_per_key": cfg["ops"],
           "ops_per_s": ops_total * steps / el, "ms_per_step": el / steps * 1e3, "steps": steps,
           "step": "lc_check_node_async (two steps in flight): host SoA -> H2D -> search -> records "
                   "(SURVEY D-1, as the N > 1 lines' value)",
           "resident": {"ops_per_s": ops_total * steps / el_r, "ms_per_step": el_r / steps * 1e3,
                        "step": "lc_check_node_device (asynchronous), the key space resident in HBM",
                        "same_records_as_pipelined": same_r},
           "t0_kernel": NN.T0_PATH_NAMES.get(int(st.t0_path)), "t0_ms_sync_step": float(st.tier0_ms),
           "t0_achieved_gbs": alg / (st.tier0_ms * 1e-3) / 1e9 if st.tier0_ms > 0 else None,
           "events": n_ev, "synth_s": round(synth_s, 2), "pack_ms": pack_s * 1e3,
           "pack_ms_warm": pack_warm_s * 1e3,
           "pack_ops_per_s": ops_total / pack_s if pack_s > 0 else None,
           "verdicts": {"valid": int((v == 1).sum()), "invalid": int((v == 0).sum()), "unknown": int((v == -1).sum())},
           "property_check": bool((v == 1).all() and (fe == -1).all())}
    del dev, buf, packed, hist
    return out


def main():
    args = parse()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr)
    if args.config is None:
        args.config = "C2" if world == 1 else "C3"
    if args.config == "C1":
        return bench_c1(args)
    if args.jepsen:
        return bench_jepsen(args)

    import numpy as np
    # torch first: liblincheck then binds the same HIP runtime (and RCCL), so
    # torch.cuda.synchronize() below also covers the library's stream
    import torch
    import torch.distributed as dist

    # Rehearsal of the N > 1 path on a one-GPU box: LC_BENCH_DEVICE=0 puts every
    # rank on cuda:0, where RCCL refuses a second rank, so the records are then
    # all-gathered on the host over gloo instead (LC_BENCH_GATHER=host).  The
    # driver's multi-GPU runs use neither: RCCL inside liblincheck, one GPU per rank.
    if os.environ.get("LC_BENCH_DEVICE"):
        local = int(os.environ["LC_BENCH_DEVICE"])
    host_gather = world > 1 and os.environ.get("LC_BENCH_GATHER", "rccl") == "host"
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo", rank=rank, world_size=world)  # rendezvous, barriers, max time: CPU only

    from lincheck import history as H
    from lincheck import parallel as P
    from lincheck.checker import Device, Packed, PinnedRecords, comm_id

    cfg = dict(CONFIGS[args.config])
    if args.keys or args.ops:
        cfg["keys"] = args.keys or cfg["keys"]
        cfg["ops"] = args.ops or cfg["ops"]
        cfg["desc"] += f" [overridden: {cfg['keys']} keys x {cfg['ops']} ops]"
    K, ops = cfg["keys"], cfg["ops"]
    strong = bool(cfg.get("strong"))
    key0 = rank * K
    shards = None
    if strong:
        # C3: a fixed key space split over the ranks by estimated cost (SURVEY
        # E-1, parallel.cost_shards: ops x concurrency x 2^crashed, heavy keys
        # by LPT).  Every key of a synthetic config has the same estimate, so
        # the shards come out as contiguous balanced ranges; a rank
        # synthesises its own keys only, run by run.
        crashed = min(20, int(round(cfg["info_rate"] * ops * 2 / 3)))
        est = np.full(cfg["keys"], float(ops * cfg["concurrency"]) * 2.0 ** crashed)
        shards = P.cost_shards(est, world)
        K = len(shards[rank])
        key0 = int(shards[rank][0]) if K else 0
    block = max(len(x) for x in shards) if strong else K  # equal all-gather blocks
    t_gen = time.perf_counter()
    runs = [(key0, K)]
    if strong and not P.contiguous(shards[rank]):
        cut = np.flatnonzero(np.diff(shards[rank]) != 1) + 1
        runs = [(int(r[0]), len(r)) for r in np.split(shards[rank], cut)]
    parts = [H.synth(n_keys=n, ops_per_key=ops, concurrency=cfg["concurrency"], info_rate=cfg["info_rate"],
                     anomaly_rate=cfg["anomaly_rate"], seed=cfg["seed"], key_base=b) for b, n in runs]
    hist = parts[0] if len(parts) == 1 else H.History.concat(parts)
    del parts
    synth_s = time.perf_counter() - t_gen
    t_pack = time.perf_counter()
    packed = Packed(hist)
    pack_s = time.perf_counter() - t_pack
    t_gen = synth_s + pack_s
    print(f"[rank {rank}] {K} keys x {ops} ops synthesised in {synth_s:.1f} s, packed in {pack_s:.2f} s",
          file=sys.stderr, flush=True)

    cid = None
    rccl_error = None
    if world > 1 and not host_gather:
        try:
            obj = [comm_id() if rank == 0 else None]
        except Exception as e:  # RCCL missing or refusing: rank 0 tells every rank
            obj = [("error", repr(e))]
        dist.broadcast_object_list(obj, src=0)
        if isinstance(obj[0], tuple):
            rccl_error = obj[0][1]
        else:
            cid = obj[0]
    torch.cuda.set_device(local)
    algo = ALGORITHMS[args.algorithm]
    try:
        dev = Device(local, budget=args.budget, comm=(rank, world, cid) if cid is not None else None, algorithm=algo,
                     path_flags=args.path_flags)
    except Exception as e:
        if cid is None:
            raise
        dev, rccl_error = None, repr(e)
    if world > 1 and not host_gather:
        # every rank must hold a communicator, else none uses one: the records
        # then go over gloo on the host, and the line says why
        ok = torch.tensor([0 if dev is None or rccl_error else 1], dtype=torch.int32)
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        if int(ok.item()) == 0:
            host_gather = True
            if rccl_error is None:
                rccl_error = "another rank's communicator failed"
            print(f"[rank {rank}] RCCL unavailable ({rccl_error}); records gathered over gloo",
                  file=sys.stderr, flush=True)
            del dev
            dev = Device(local, budget=args.budget, algorithm=algo, path_flags=args.path_flags)
    n_node = block * (1 if host_gather else world)
    node_buf = np.zeros(max(n_node, 1), np.uint64)

    def barrier():
        if world > 1:
            dist.barrier()

    def sync():
        dev.wait()
        torch.cuda.synchronize()

    def node_records(rec):
        if not host_gather:
            return rec
        parts = [None] * world
        dist.all_gather_object(parts, rec.copy())
        return np.concatenate(parts)

    # ---- D-1: host SoA -> node verdict records.  The timed steps are the
    # pipelined call (lc_check_node_async: each step's upload overlaps the
    # search of the step before, records land in page-locked memory); the
    # synchronous call (lc_check_node, one step at a time) runs after them
    # for its own rate and for the per-launch kernel times of the roofline.
    d1_t0, d1_t3, d1_t3b, d1_wgl = [], [], [], []
    d1_path = {}  # the register tier's kernel and event word width (lc_stats, synchronous steps)
    pipelined = not args.d1_sync
    node_pin = PinnedRecords(n_node) if pipelined else None

    def record(st):
        d1_path["t0_path"], d1_path["ev_word_bytes"] = int(st.t0_path), int(st.ev_word_bytes)
        d1_t0.append(st.tier0_ms if st.tier0_ms > 0 else st.kernel_ms)
        if st.tier3_ms > 0:
            d1_t3.append(st.tier3_ms)
            d1_t3b.append(st.t3_bytes)
        if st.wgl_ms > 0:
            d1_wgl.append(st.wgl_ms)

    def d1_step():
        rec, st = dev.check_node(packed, block, out=node_buf)
        record(st)
        return rec

    n_enq = [0]

    def d1_pipe_step():
        enq, st = dev.check_node_async(packed, block, node_pin)
        if enq:
            n_enq[0] += 1
        else:
            record(st)
        return node_pin[:n_node]

    def timed(step):
        for _ in range(args.warmup):
            step()
        sync(); barrier(); sync()
        del d1_t0[:], d1_t3[:], d1_t3b[:], d1_wgl[:]
        n_enq[0] = 0
        t0 = time.perf_counter()
        for i in range(args.steps):
            ts = time.perf_counter()
            rec = step()
            if time.perf_counter() - ts > 10.0:  # (long steps: a sign of life for the job's watchdog)
                print(f"[rank {rank}] step {i + 1}/{args.steps}: {time.perf_counter() - ts:.1f} s", file=sys.stderr,
                      flush=True)
        sync(); barrier(); sync()
        el = time.perf_counter() - t0
        if world > 1:
            t = torch.tensor([el], dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = float(t.item())
        return el, np.array(rec, copy=True)

    d1_sync = None
    if pipelined:
        elapsed, rec = timed(d1_pipe_step)
        n_pipe = n_enq[0]
        el_s, rec_s = timed(d1_step)
        d1_sync = {"ms_per_step": el_s / args.steps * 1e3, "elapsed_s": el_s,
                   "pipelined_steps": n_pipe, "same_records": bool(np.array_equal(rec, rec_s))}
    else:
        elapsed, rec = timed(d1_step)
    node = node_records(rec.copy())

    # ---- resident shard: steps only enqueued, exchange on the library stream
    resident = None
    if not args.no_resident:
        db = dev.upload(packed)
        for _ in range(args.warmup):
            db.check_node(block, asynchronous=True)
        sync(); barrier(); sync()
        tr = time.perf_counter()
        t3 = []
        for _ in range(args.steps):
            st = db.check_node(block, asynchronous=True)
            if st.tier3_ms > 0:
                t3.append(st.tier3_ms)
        n_async, span_ms = dev.wait()
        sync(); barrier(); sync()
        el_r = time.perf_counter() - tr
        if world > 1:
            t = torch.tensor([el_r], dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el_r = float(t.item())
        same = bool(np.array_equal(dev.node_records(block * (1 if host_gather else world)),
                                   rec[:block * (1 if host_gather else world)]))
        total_ops = (cfg["keys"] if strong else K * world) * ops
        resident = {"ops_per_s": total_ops * args.steps / el_r, "ms_per_step": el_r / args.steps * 1e3,
                    "async_steps": n_async, "tier0_ms_per_launch": (span_ms / n_async) if n_async else None,
                    "tier3_ms": float(np.mean(t3)) if t3 else None, "same_records_as_d1": same}
        del db

    probes = probes_t3 = None
    if rank == 0 and not args.no_probes and args.algorithm == "linear":
        # probe count from one extra pass with
        # LC_OPT_COUNT_PROBES: the timed steps skip the per-event popcounts
        dev_c = Device(local, budget=args.budget, count_probes=True)
        pst = dev_c.upload(packed).check(peak=False).stats
        probes, probes_t3 = pst["probes"], pst["probes_t3"]
        del dev_c

    if rank == 0:
        if not strong:
            shards = [np.arange(r * K, (r + 1) * K) for r in range(world)]
        # the node's verdicts from its gathered blocks (rank order, padding 0),
        # back in the key space's order
        nv, _, nfe = P.node_key_order(node, shards, block)
        v_host, fe_host = nv[shards[0]], nfe[shards[0]]  # rank 0's own shard
        n_keys_total = int(nv.size)
        decided = int(((nv == 1) | (nv == 0)).sum())
        # ops checked: every op of a key that reached a verdict (valid or
        # invalid); a key that ends :unknown (budget) was not checked
        ops_total = (cfg["keys"] if strong else K * world) * ops
        ops_checked = decided * ops
        # `value`: SURVEY D-1's host-link-inclusive step (packed host SoA ->
        # verdict records in host memory, pipelined), K steps between
        # barriers, max over ranks.  The resident step (the shard already in
        # HBM) is reported beside it in `resident` and is never `value`.
        el_pipe = elapsed
        value = ops_checked * args.steps / elapsed
        if resident:
            resident["ops_checked_per_s"] = ops_checked * args.steps / (resident["ms_per_step"] * args.steps * 1e-3)
        d1_pipelined = None
        if pipelined:
            d1_pipelined = {"ms_per_step": el_pipe / args.steps * 1e3, "ops_per_s": ops_checked * args.steps / el_pipe,
                            "what": "lc_check_node_async, two steps in flight: packed host SoA -> H2D -> search -> "
                                    "verdict records in page-locked host memory (host-link inclusive)"}
        if d1_sync is not None:
            d1_sync["ops_per_s"] = ops_checked * args.steps / d1_sync["elapsed_s"]
        avg_t0 = float(np.mean(d1_t0)) if d1_t0 else 0.0
        # the register tier's launch time: the resident steps' HIP-event span
        # per launch when they ran (one launch per step); the synchronous
        # steps' per-launch time otherwise (a large shard's synchronous step is
        # four chunk launches waiting on their uploads: not a launch time)
        t0_src = "synchronous D-1 steps (HIP events)"
        if resident and resident.get("tier0_ms_per_launch") and not d1_t3:
            avg_t0 = float(resident["tier0_ms_per_launch"])
            t0_src = "resident asynchronous steps (HIP-event span / launches)"
        avg_t3 = float(np.mean(d1_t3)) if d1_t3 else 0.0
        n_events = int(packed.ev_off[-1])
        max_events = int(np.diff(packed.ev_off.astype(np.int64)).max()) if K else 0
        # Algorithmic HBM bytes of one launch of the dominant kernel (DESIGN.md
        # section 3): T0 reads every event word once (2 B when the 16-bit
        # words are read in place, as k_spec does, else 4 B), the key offsets
        # (8 B) and LPT order (4 B), the transition table once, and writes a
        # verdict record (8 B) per key.
        from lincheck import _native as NN
        ewb = d1_path.get("ev_word_bytes") or 4
        alg_bytes = ewb * n_events + 8 * (K + 1) + 4 * K + 4 * int(packed.view.n_trans) + 8 * K
        kt = avg_t0
        t0_name = NN.T0_PATH_NAMES.get(d1_path.get("t0_path", 1), "T0")
        dominant = f"T0 register tier ({t0_name})"
        d4_t3 = None
        if avg_t3 > avg_t0:
            # the HBM tier dominates (C4).  Its layered form (k_search_layers)
            # touches HBM only to stream the config-set arrays: 8 B per entry
            # read or written (lc_stats.t3_bytes, counted by the kernel).
            # SURVEY D-4's notional 64 B line per hash probe is kept beside it
            # (d4_model_gbs) -- the config-keyed T3 moved about that much.
            dominant = "k_search_layers (T3L)"
            alg_bytes = int(np.mean(d1_t3b)) if d1_t3b else 0
            kt = avg_t3
            if probes_t3:
                d4_t3 = 64 * probes_t3 / (kt * 1e-3) / 1e9
        wgl = None
        avg_wgl = float(np.mean(d1_wgl)) if d1_wgl else 0.0
        if args.algorithm != "linear":
            # knossos.wgl's walk (k_wgl) and what it moved: one batch check
            # for the per-key cache sizes and the walk's steps
            wres = dev.check(packed) if world == 1 else None
            wsel = (wres.analyzer == 1) if wres is not None else None
            cache_entries = int(wres.peak[wsel].sum()) if wres is not None else None
            wsteps = int(wres.stats["wgl_steps"]) if wres is not None else None
            wgl = {"ms_per_launch": avg_wgl, "launches": len(d1_wgl),
                   "keys_answered": int(wsel.sum()) if wsel is not None else None,
                   "keys_decided": int(((wres.valid != -1) & wsel).sum()) if wsel is not None else None,
                   "keys_spilled": int(wres.stats["wgl_spilled"]) if wres is not None else None,
                   "steps": wsteps, "cache_entries": cache_entries,
                   "probes": int(wres.stats["probes"]) if wres is not None else None,
                   "steps_per_s": (wsteps / (avg_wgl * 1e-3)) if wsteps and avg_wgl > 0 else None}
            if wres is not None and wsel.any():
                # the walk is serial per key (one wave each): the launch lasts
                # as long as its longest walk, whose cache size (steps down)
                # the records hold
                pk = wres.peak[wsel].astype(np.int64)
                wgl["cache_per_key"] = {"max": int(pk.max()), "median": float(np.median(pk)),
                                        "max_share_of_all": float(pk.max() / max(1, pk.sum()))}
            if args.algorithm == "wgl" or avg_wgl >= max(avg_t0, avg_t3):
                # Algorithmic bytes of a WGL launch: the event words (4 B),
                # each cache entry written once (32 B), an 80-B frame written
                # or read per step, the records -- the probes' reads come on
                # top (up to a window of 32-B entries per step).
                dominant = "k_wgl (knossos.wgl walk)"
                kt = avg_wgl
                alg_bytes = 4 * n_events + 32 * (cache_entries or 0) + 80 * (wsteps or 0) + 8 * K
                tags = ("k_wgl",)
        achieved = alg_bytes / (kt * 1e-3) / 1e9 if kt > 0 else 0.0
        # measured HBM traffic and VALU issue of the same kernel on the same
        # workload, from the committed rocprofv3 --pmc summaries (profiles/)
        traffic = traffic_src = issue = None
        if "k_wgl" not in dominant:
            tags = (t0_name,) if "T0" in dominant else ("k_search_layers",)
        refused = []
        for fpath in sorted(glob.glob(os.path.join(ROOT, "profiles", "*.json"))):
            try:
                d = json.load(open(fpath))
            except (OSError, ValueError):
                continue
            if not isinstance(d, dict):
                continue
            kname = d.get("kernel") or ""
            if (d.get("workload") != args.config or d.get("budget", args.budget) != args.budget
                    or d.get("round") != PROFILE_ROUND or d.get("algorithm", "linear") != args.algorithm
                    or not any(t in kname for t in tags)):
                continue
            # counters of the launch this line divides by, and nothing else:
            # the same key count, and whole launches only (tools/
            # profile_summary.py keeps the dispatches of the largest grid; a
            # chunk launch of a large shard's synchronous step is not one)
            why = profile_mismatch(d, K, kname)
            if why:
                refused.append({"file": os.path.basename(fpath), "why": why})
                continue
            if d.get("bytes_per_launch"):
                traffic, traffic_src = d["bytes_per_launch"], os.path.basename(fpath)
            if d.get("sq_insts_valu_per_launch") and kt > 0:
                # VALU issue capacity over the launch: every SIMD issues one
                # wave64 VALU instruction per 2 cycles (MI355X_MICROARCH.md)
                import torch as _t
                simds = 4 * _t.cuda.get_device_properties(local).multi_processor_count
                cap = simds * SHADER_CLOCK_HZ / 2 * kt * 1e-3
                issue = {"valu_per_launch": d["sq_insts_valu_per_launch"], "capacity": cap,
                         "frac": d["sq_insts_valu_per_launch"] / cap, "simds": simds,
                         "clock_ghz": SHADER_CLOCK_HZ / 1e9, "source": os.path.basename(fpath),
                         "grid_size": d.get("grid_size"), "waves_per_launch": d.get("sq_waves_per_launch")}
        nproc, aff, quota = host_cores()
        cpu = parity = None
        if world == 1 and not args.no_cpu:
            cpu, parity = cpu_baseline(args, cfg, K, key0, hist, ops, v_host, fe_host, nproc, aff, quota)
        c3 = None
        if world == 1 and args.config == "C2" and not (args.no_c3 or args.keys or args.ops):
            c3 = bench_c3_strong(args, local)
        line = {
            "metric": METRIC,
            "value": value,
            "unit": "ops/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "strong" if strong else "weak",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic",
            "config": {"workload": cfg["desc"], "keys_total": n_keys_total, "keys_per_gpu": K, "ops_per_key": ops,
                       "concurrency": cfg["concurrency"], "budget": args.budget, "algorithm": args.algorithm,
                       "parallelism": f"keys sharded over {world} GPU(s), records all-gathered "
                                      f"({('host/gloo, RCCL unavailable: ' + rccl_error) if rccl_error else 'host/gloo rehearsal' if host_gather else 'RCCL' if world > 1 else 'one rank'})"},
            "step": (("lc_check_node_async (two steps in flight)" if pipelined else "lc_check_node") +
                     ": packed host SoA -> H2D -> search -> verdict records -> all-gather -> host (SURVEY D-1)"),
            "d1_pipelined": d1_pipelined,
            "d1_sync": d1_sync,
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "kernel": dominant,
                         "alg_bytes_per_launch": alg_bytes, "avg_launch_ms": kt, "event_word_bytes": ewb,
                         "traffic_over_alg": (traffic / alg_bytes) if traffic and alg_bytes else None,
                         "traffic_source": traffic_src, "issue": issue, "launch_time_from": t0_src,
                         "launches": len(d1_t0), "d4_model_gbs": d4_t3},
            "cpu_baseline": cpu,
            "ops_total": ops_total,
            "ops_checked_per_step": ops_checked,
            "keys_to_verdict_per_s": decided * args.steps / elapsed,
            # every key ends with a :valid? (true / false / :unknown at the
            # budget): the rate at which the step answers for all of them
            "ops_answered_per_s": ops_total * args.steps / elapsed,
            "resident": resident,
            "tier0_ms": avg_t0,
            "tier3_ms": avg_t3,
            "wgl": wgl,
            "probes": probes,
            "probes_t3": probes_t3,
            # hash-probe throughput (north_star; SURVEY D-4): the oracle's
            # probe count of the tier over that tier's launch time
            "probes_per_s": probe_rates(probes, probes_t3, avg_t0, avg_t3, d1_t3, wgl),
            "profiles_refused": refused or None,
            "ns_per_event_critical_path": avg_t0 * 1e6 / max(max_events, 1),
            "verdicts": {"valid": int((nv == 1).sum()), "invalid": int((nv == 0).sum()),
                         "unknown": int((nv == -1).sum())},
            "parity_vs_oracle": parity,
            "setup_s": round(t_gen, 2),
            "synth_s": round(synth_s, 2),
            "pack_ms": pack_s * 1e3,
            "pack_ops_per_s": K * ops / pack_s if pack_s > 0 else None,
            "c3_strong": c3,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
