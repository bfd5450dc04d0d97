"""lc_pack on the box's host cores:
the key-major path against the bucketing path (LC_PACK_GENERAL) on C5 and
C3 shapes, first (fresh memory) and warm packs; plus the host -> device
copy rate of pageable and page-locked memory (what a device-side pack from
the raw history columns would pay to get them there).

    python tools/pack_timing.py [--c3-keys 100000] > gpurun_out/pack_timing.json
"""

import argparse
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "jepsen-etcd-demo_amd"))

import numpy as np  # noqa: E402

try:  # torch first: the library then binds torch's HIP runtime (as bench.py does)
    import torch  # noqa: F401
except ImportError:
    pass
from lincheck import _native as N  # noqa: E402
from lincheck import history as H  # noqa: E402


def digest(handle):
    """A hash of the packed arrays the device reads (the 32-bit words widened
    from the 16-bit ones where only those are given)."""
    import hashlib
    v = N.LcBatch()
    N.check(N.lib().lc_packed_view(handle, C.byref(v)))
    K = int(v.n_keys)
    ev_off = np.ctypeslib.as_array(v.ev_off, shape=(K + 1,))
    n = int(ev_off[-1])
    hsh = hashlib.sha256()
    hsh.update(ev_off.tobytes())
    if v.events16:
        e16 = np.ctypeslib.as_array(v.events16, shape=(n,))
        hsh.update(b"16" + e16.tobytes())
    else:
        hsh.update(b"32" + np.ctypeslib.as_array(v.events, shape=(n,)).tobytes())
    hsh.update(np.ctypeslib.as_array(v.trans, shape=(int(v.n_trans),)).tobytes())
    hsh.update(np.ctypeslib.as_array(v.key_width, shape=(K,)).tobytes())
    hsh.update(np.ctypeslib.as_array(v.key_states, shape=(K,)).tobytes())
    return hsh.hexdigest()[:16]


def pack_ms(h, flags, reps):
    c = h.as_c()
    out = []
    dg = None
    for i in range(reps):
        o = N.LcPackOpts(0)
        o.flags = flags
        handle = C.c_void_p()
        t = time.perf_counter()
        N.check(N.lib().lc_pack(C.byref(c), C.byref(o), C.byref(handle)))
        out.append((time.perf_counter() - t) * 1e3)
        path = N.lib().lc_packed_path(handle)
        if i == 0:
            dg = digest(handle)
        N.lib().lc_packed_free(handle)
    return {"first_ms": out[0], "warm_ms": min(out[1:]) if len(out) > 1 else None, "path": path, "all_ms": out,
            "digest": dg}


def h2d_rates():
    try:
        import torch
        if not torch.cuda.is_available():
            return None
    except ImportError:
        return None
    res = {}
    n = 1 << 30
    src = torch.empty(n, dtype=torch.uint8).fill_(1)
    pin = torch.empty(n, dtype=torch.uint8).pin_memory().fill_(1)
    dst = torch.empty(n, dtype=torch.uint8, device="cuda")
    for name, s in (("pageable", src), ("pinned", pin)):
        dst.copy_(s)
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(3):
            dst.copy_(s)
        torch.cuda.synchronize()
        res[name + "_gbs"] = 3 * n / (time.perf_counter() - t) / 1e9
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--c3-keys", type=int, default=100_000)
    args = ap.parse_args()
    out = {"threads_cap": 16, "nproc": os.cpu_count()}
    h5 = H.synth(n_keys=1000, ops_per_key=1000, concurrency=10, anomaly_rate=0.05, seed=5)
    out["C5"] = {"rows": len(h5),
                 "key_major": pack_ms(h5, 0, 8), "bucketing": pack_ms(h5, N.LC_PACK_GENERAL, 4)}
    out["C5"]["same_arrays"] = out["C5"]["key_major"]["digest"] == out["C5"]["bucketing"]["digest"]
    print(json.dumps(out), flush=True)
    del h5
    t = time.perf_counter()
    h3 = H.synth(n_keys=args.c3_keys, ops_per_key=2000, concurrency=10, seed=3)
    out["C3"] = {"keys": args.c3_keys, "synth_s": time.perf_counter() - t,
                 "key_major": pack_ms(h3, 0, 3), "bucketing": pack_ms(h3, N.LC_PACK_GENERAL, 2)}
    out["C3"]["same_arrays"] = out["C3"]["key_major"]["digest"] == out["C3"]["bucketing"]["digest"]
    print(json.dumps(out), flush=True)
    del h3
    out["h2d"] = h2d_rates()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
