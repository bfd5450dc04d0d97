"""Ablation timing of the device search (diagnostic, not a test)."""
import sys, time
import numpy as np
from lincheck import history as H
from lincheck.checker import Device, Packed

h = H.synth(n_keys=1000, ops_per_key=1000, concurrency=10, seed=2)
import sys
sys.path.insert(0, "../oracle")
import linear_ref as LR
ops = H.synth(n_keys=20, ops_per_key=1000, concurrency=10, seed=2).to_ops()
from collections import Counter
cnt = Counter()
for k in range(20):
    _o, evs = LR.complete(LR.subhistory(ops, k))
    n = 0
    for kind, _, _ in evs:
        if kind == "invoke": n += 1
        else: cnt[n] += 1; n -= 1
print("pending at ok:", sorted(cnt.items()))
pk = Packed(h)
for mode, peak in ((1, False), (5, False), (0, False)):
    dev = Device(0, debug_mode=mode)
    db = dev.upload(pk)
    for _ in range(3):
        r = db.check(peak)
    ts = [db.check(peak).stats["kernel_ms"] for _ in range(10)]
    print(f"mode {mode} peak {peak}: kernel {np.median(ts):.3f} ms  deep {r.stats['deep_keys']}", flush=True)
