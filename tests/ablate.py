"""Ablation timing of the device search (diagnostic, not a test)."""
import sys, time
import numpy as np
from lincheck import history as H
from lincheck.checker import Device, Packed

h = H.synth(n_keys=1000, ops_per_key=1000, concurrency=10, seed=2)
pk = Packed(h)
for mode in (1, 3, 4, 0):
    dev = Device(0, debug_mode=mode)
    db = dev.upload(pk)
    for _ in range(3):
        r = db.check()
    ts = [db.check().stats["kernel_ms"] for _ in range(10)]
    print(f"mode {mode}: kernel {np.median(ts):.3f} ms  deep {r.stats['deep_keys']}", flush=True)
