"""Benchmark: history ops linearizability-checked per second (BASELINE.json metric).

One step = one pass of the device search (liblincheck.so, lc_check_device)
over one batch of synthetic cas-register histories already resident in HBM,
with the per-key verdict records left on the device and, for N > 1,
all-gathered across ranks over RCCL (the one exchange step of the path,
SURVEY.md 8(e)).

Workload (N=1 = BASELINE.json configs[1], "C2"): 1,000 keys x 1,000 client
ops, concurrency 10, cas-register over values 0..4 (etcdemo.clj:67-69),
seed 2.  Weak scaling: rank r checks keys [r*1000, (r+1)*1000) of the same
seeded key space, so per-GPU work is fixed as N grows.

Also reported (one JSON line on rank 0):
  roofline      the search kernels' algorithmic HBM bytes per launch over
                their HIP-event time (DESIGN.md "Measurement"), MI355X
                peak 8 TB/s; traffic from profiles/*pmc*.json if committed.
  cpu_baseline  the C restatement of knossos.linear (oracle/linear_ref.c,
                kind "port") on this host's cores, same workload (rank 0, N=1).
"""

import argparse
import glob
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for p in (os.path.join(ROOT, "jepsen-etcd-demo_amd"), os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec

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
    ap.add_argument("--config", default="C2", choices=sorted(CONFIGS))
    ap.add_argument("--budget", type=int, default=1 << 20)
    ap.add_argument("--no-cpu", action="store_true",
                    help="skip the CPU baseline and the host-to-host pass (profiling runs: only the timed steps "
                         "and the probe-count pass launch the search)")
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--keys", type=int, default=0, help="override keys per GPU (exploration only)")
    ap.add_argument("--ops", type=int, default=0, help="override ops per key (exploration only)")
    return ap.parse_args()


def bench_c1(args):
    """C1 (BASELINE.json configs[0]): the demo's check phase end to end, as
    etcdemo.clj:115-119 runs it -- history.edn on disk -> lc_edn_read ->
    independent/checker over compose {:linear linearizable, :timeline} ->
    the result map.  A step is that whole call; the latency to a verdict,
    not the kernel, is what this config measures."""
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
        "metric": "history ops linearizability-checked/sec (whole node)",
        "value": n_ops * args.steps / elapsed, "unit": "ops/s", "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u64", "data": "synthetic",
        "config": {"workload": CONFIGS["C1"]["desc"], "keys_per_gpu": 6, "ops_per_key": 100, "concurrency": 10,
                   "budget": args.budget, "parallelism": "1 GPU (latency case)"},
        "roofline": None,
        "cpu_baseline": cpu,
        "step": "lc_edn_read + independent/checker(compose(linearizable, timeline)) -> result map",
        "valid?": out["valid?"], "failures": out["failures"], "parity_vs_oracle": parity,
    }
    print(json.dumps(line, default=str), flush=True)


def main():
    args = parse()
    if args.config == "C1":
        return bench_c1(args)
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr)

    import numpy as np
    import torch
    import torch.distributed as dist

    # Rehearsal of the N > 1 path on a one-GPU box: LC_BENCH_BACKEND=gloo and
    # LC_BENCH_DEVICE=0 put every rank on cuda:0 (RCCL refuses two ranks on one
    # device).  The driver's multi-GPU runs use neither: RCCL, one GPU per rank.
    backend = os.environ.get("LC_BENCH_BACKEND", "nccl")
    if os.environ.get("LC_BENCH_DEVICE"):
        local = int(os.environ["LC_BENCH_DEVICE"])
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend, rank=rank, world_size=world)
    else:
        torch.cuda.set_device(local)

    from lincheck import history as H
    from lincheck import _native as N
    from lincheck.checker import Device, Packed

    cfg = dict(CONFIGS[args.config])
    if args.keys or args.ops:
        cfg["keys"] = args.keys or cfg["keys"]
        cfg["ops"] = args.ops or cfg["ops"]
        cfg["desc"] += f" [overridden: {cfg['keys']} keys x {cfg['ops']} ops]"
    K, ops = cfg["keys"], cfg["ops"]
    strong = bool(cfg.get("strong"))
    key0 = rank * K
    if strong:  # C3: a fixed key space split over the ranks (contiguous, equal shards)
        key0 = rank * K // world
        K = (rank + 1) * K // world - key0
    t_gen = time.time()
    hist = H.synth(n_keys=K, ops_per_key=ops, concurrency=cfg["concurrency"], info_rate=cfg["info_rate"],
                   anomaly_rate=cfg["anomaly_rate"], seed=cfg["seed"], key_base=key0)
    print(f"[rank {rank}] synthesised {K} keys x {ops} ops in {time.time() - t_gen:.1f} s", file=sys.stderr, flush=True)
    packed = Packed(hist)
    t_gen = time.time() - t_gen
    dev = Device(local, budget=args.budget)
    db = dev.upload(packed)
    print(f"[rank {rank}] packed + uploaded; setup {t_gen:.1f} s", file=sys.stderr, flush=True)

    # device-resident result arrays (torch tensors) -> no D2H inside the step.
    # Two sets, alternating per step: step k's records are packed and
    # all-gathered on torch's stream while step k+1's search (the library's
    # own stream) writes the other set; before a set is reused, the event
    # recorded after its packing is waited on.
    tdev = torch.device("cuda", local)
    import ctypes as C
    bufs = []
    for _ in range(2 if world > 1 else 1):
        valid = torch.empty(K, dtype=torch.int8, device=tdev)
        fail_event = torch.empty(K, dtype=torch.int32, device=tdev)
        cause = torch.empty(K, dtype=torch.uint8, device=tdev)
        # verdict records only: no peak sizes, no counterexample configs in the step
        res = N.LcResult(C.cast(valid.data_ptr(), N.P(C.c_int8)), C.cast(fail_event.data_ptr(), N.P(C.c_int32)),
                         C.cast(cause.data_ptr(), N.P(C.c_uint8)), None, None, None)
        bufs.append({"valid": valid, "fail_event": fail_event, "cause": cause, "res": res, "packed": None})
    # equal-sized all-gather blocks: a strong-scaling shard may be one key short
    K_blk = -(-cfg["keys"] // world) if strong else K
    gathered = torch.empty(K_blk * world, dtype=torch.int64, device=tdev) if world > 1 else None
    rec = torch.zeros(K_blk, dtype=torch.int64, device=tdev) if world > 1 else None

    from lincheck import parallel as P

    n_step = [0]
    # A step whose keys all stay in the register tier is only enqueued
    # (LC_DEV_ASYNC), so step k+1's launch is queued while step k runs; the
    # HIP events of lc_wait give the launches' span.  N > 1: step k's records
    # are packed and all-gathered during step k+1, once lc_wait_step has seen
    # step k's search finish (step k+1's search keeps running); the last
    # step's exchange is flushed inside the timed region.
    pending = [None]  # result set whose search is enqueued, records not yet exchanged

    def exchange(b, back):  # the path's one exchange step: verdict records over RCCL
        dev.wait_step(back)
        rec[:K] = P.pack_records(b["valid"], b["cause"], b["fail_event"])
        b["packed"] = torch.cuda.Event()
        b["packed"].record()
        dist.all_gather_into_tensor(gathered, rec)

    def step():
        b = bufs[n_step[0] % len(bufs)]
        n_step[0] += 1
        if b["packed"] is not None:
            b["packed"].synchronize()  # this set's previous records are packed
        st = db.check_into(b["res"], asynchronous=True)
        if world > 1:
            if pending[0] is not None:
                exchange(pending[0], 1)  # the previous step's search
            pending[0] = b
        return st

    def flush():
        if world > 1 and pending[0] is not None:
            exchange(pending[0], 0)
            pending[0] = None

    for _ in range(args.warmup):
        step()
    flush()
    torch.cuda.synchronize()
    dev.wait()  # resets the asynchronous-step span
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    kernel_ms, tier0_ms, tier3_ms, probes, deep = [], [], [], 0, 0
    t0 = time.perf_counter()
    for _ in range(args.steps):
        st = step()
        kernel_ms.append(st.kernel_ms)
        tier0_ms.append(st.tier0_ms)
        tier3_ms.append(st.tier3_ms)
        deep = st.deep_keys
    flush()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    n_async, span_ms = dev.wait()
    if n_async:  # asynchronous steps: per-launch time = the span over the launches
        assert n_async == args.steps, (n_async, args.steps)
        kernel_ms = tier0_ms = [span_ms / n_async]
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=tdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # results of the last step (host copy, outside the timed region)
    last = bufs[(n_step[0] - 1) % len(bufs)]
    v_host = last["valid"].cpu().numpy()
    fe_host = last["fail_event"].cpu().numpy()
    node = None
    if world > 1:
        # whole-node verdicts from the last step's all-gather (the rank blocks
        # are K_blk records each; a short strong-scaling shard leaves padding)
        torch.cuda.synchronize()
        g = gathered.cpu().numpy().reshape(world, K_blk)
        parts = []
        for r in range(world):
            kr = ((r + 1) * cfg["keys"] // world - r * cfg["keys"] // world) if strong else K
            parts.append(g[r, :kr])
        gv, _, gfe = P.unpack_records(np.concatenate(parts))
        # rank 0's block of the gather must be exactly its local records
        own_ok = bool(np.array_equal(gv[:K], v_host) and np.array_equal(gfe[:K], fe_host))
        node = {"keys": int(gv.size), "valid": int((gv == 1).sum()), "invalid": int((gv == 0).sum()),
                "unknown": int((gv == -1).sum()), "rank0_block_matches_local": own_ok}
    h2h_ms, h2h_same = None, None
    if rank == 0 and not args.no_cpu:
        # SURVEY.md 8(d) D-1's end-to-end rate, outside the timed region: one
        # lc_check_batch from the packed SoA in host memory to host verdict
        # arrays (upload over PCIe + search + download), best of 3.  Never `value`.
        h2h = []
        for _ in range(3):
            th = time.perf_counter()
            hr = dev.check(packed, verdicts_only=True)
            h2h.append(time.perf_counter() - th)
        h2h_ms = min(h2h) * 1e3
        h2h_same = bool(np.array_equal(hr.valid, v_host) and np.array_equal(hr.fail_event, fe_host))
    if rank == 0:
        # probe count from one extra, untimed pass with
        # LC_OPT_COUNT_PROBES: the timed steps skip the per-event popcounts
        dev_c = Device(local, budget=args.budget, count_probes=True)
        pst = dev_c.upload(packed).check(peak=False).stats
        probes, probes_t3 = pst["probes"], pst["probes_t3"]
        del dev_c

    if rank == 0:
        n_ops_total = (cfg["keys"] if strong else K * world) * ops
        value = n_ops_total * args.steps / elapsed
        avg_kernel_ms = float(np.mean(kernel_ms))
        avg_t0_ms = float(np.mean(tier0_ms))
        n_events = int(packed.ev_off[-1])
        max_events = int(np.diff(packed.ev_off.astype(np.int64)).max()) if K else 0
        # Algorithmic HBM bytes of one launch of the dominant kernel (the
        # register-lattice tier, DESIGN.md "Measurement"): every event word
        # (4 B), the key offsets (8 B) and LPT order (4 B) read, the
        # transition table read once, a verdict record (valid 1 B + failing
        # event 4 B + cause 1 B) written per key.
        alg_bytes = 4 * n_events + 8 * (K + 1) + 4 * K + 4 * int(packed.view.n_trans) + 6 * K
        achieved = alg_bytes / (avg_t0_ms * 1e-3) / 1e9
        dominant = "k_search_lattice (T0)"
        avg_t3_ms = float(np.mean(tier3_ms))
        if avg_t3_ms > avg_t0_ms:
            # The HBM tier dominates (deep keys, C4): its algorithmic traffic
            # is SURVEY.md 8(d) D-4's one 64 B line per hash probe, counted
            # for that tier alone, over the span of its launches.
            dominant = "k_search_hbm (T3)"
            alg_bytes = 64 * probes_t3
            achieved = alg_bytes / (avg_t3_ms * 1e-3) / 1e9
        # SURVEY.md 8(d) D-4's notional model (16 B A3 record per op, 17 B per
        # key, one 64 B HBM line per probe) for comparison only: in T0 the
        # probes never leave registers.
        d4_bytes = 16 * K * ops + 17 * K + 64 * probes
        traffic = None
        for fpath in sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc*.json"))):
            try:
                d = json.load(open(fpath))
                if (d.get("workload") == args.config and d.get("bytes_per_launch")
                        and d.get("budget", args.budget) == args.budget):
                    traffic = d["bytes_per_launch"]
            except (OSError, ValueError):
                pass
        cpu = None
        parity = None
        if world == 1 and not args.no_cpu:
            import cref
            threads = args.cpu_threads or min(16, os.cpu_count() or 1)

            def first_keys(k):  # the batch's first k keys (per-key seeded generator)
                if k == K:
                    return hist
                return H.synth(n_keys=k, ops_per_key=ops, concurrency=cfg["concurrency"], info_rate=cfg["info_rate"],
                               anomaly_rate=cfg["anomaly_rate"], seed=cfg["seed"], key_base=key0)

            # Bounded sample (~20 s of CPU work): time one key per thread,
            # then take as many of the batch's first keys as fit.
            kp = min(K, threads)
            tc = time.perf_counter()
            keys, orc = cref.check_history(first_keys(kp).as_c(), budget=args.budget, threads=threads)
            tcpu = time.perf_counter() - tc
            ks = kp
            if kp < K:
                ks = K if tcpu * K / kp <= 20.0 else min(K, max(kp, int(kp * 20.0 / max(tcpu, 1e-6)) // kp * kp))
                if ks > kp:
                    tc = time.perf_counter()
                    keys, orc = cref.check_history(first_keys(ks).as_c(), budget=args.budget, threads=threads)
                    tcpu = time.perf_counter() - tc
            # one thread on ~1/8 of that sample
            k1 = max(1, ks // 8)
            t1 = time.perf_counter()
            cref.check_history(first_keys(k1).as_c(), budget=args.budget, threads=1)
            t1 = time.perf_counter() - t1
            what = (f"full {args.config} batch ({K} keys x {ops} ops)" if ks == K
                    else f"first {ks} of the {K} keys of the {args.config} batch ({ops} ops each)")
            cpu = {"value": ks * ops / tcpu, "unit": "ops/s", "cores": threads, "kind": "port",
                   "sample": f"{what}, oracle/linear_ref.c, {threads} threads, {tcpu:.2f} s",
                   "one_thread": {"value": k1 * ops / t1, "cores": 1,
                                  "sample": f"first {k1} keys of the batch, 1 thread, {t1:.2f} s"}}
            parity = bool(np.array_equal(orc["valid"], v_host[:ks]) and np.array_equal(orc["fail_event"], fe_host[:ks]))
            if ks < K:
                cpu["parity_sample_keys"] = ks
        line = {
            "metric": "history ops linearizability-checked/sec (whole node)",
            "value": value,
            "unit": "ops/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "strong" if strong else "weak",
            "vs_baseline": None,
            "dtype": "u64",
            "data": "synthetic",
            "config": {"workload": cfg["desc"], "keys_per_gpu": K, "ops_per_key": ops,
                       "concurrency": cfg["concurrency"], "budget": args.budget,
                       "parallelism": f"keys sharded over {world} GPU(s)"},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "kernel": dominant,
                         "alg_bytes_per_launch": alg_bytes},
            "cpu_baseline": cpu,
            "kernel_ms": avg_kernel_ms,
            "tier0_ms": avg_t0_ms,
            "tier3_ms": avg_t3_ms,
            "probes_t3": probes_t3,
            "ns_per_event_critical_path": avg_t0_ms * 1e6 / max(max_events, 1),
            "probes_per_s": probes / (avg_kernel_ms * 1e-3),
            "d4_model_gbs": d4_bytes / (avg_kernel_ms * 1e-3) / 1e9,
            "deep_keys": deep,
            "verdicts": {"valid": int((v_host == 1).sum()), "invalid": int((v_host == 0).sum()),
                         "unknown": int((v_host == -1).sum())},
            "parity_vs_oracle": parity,
            "node_verdicts": node,
            "host_to_host": None if h2h_ms is None else {
                "ms": h2h_ms, "ops_per_s_one_gpu": K * ops / (h2h_ms * 1e-3), "same_verdicts_as_resident": h2h_same,
                "what": "rank 0: lc_check_batch from packed host SoA to host verdicts (PCIe incl.), best of 3"},
            "setup_s": round(t_gen, 2),
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
