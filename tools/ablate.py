"""Ablation timing of T0 (diagnostic): debug_mode 1 = event bookkeeping only."""
import os, sys
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(root, "jepsen-etcd-demo_amd")]
import numpy as np
from lincheck import history as H
from lincheck.checker import Device, Packed
keys = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
h = H.synth(n_keys=keys, ops_per_key=1000, concurrency=10, seed=2)
pk = Packed(h)
for mode in (1, 0):
    dev = Device(0, debug_mode=mode)
    db = dev.upload(pk)
    for _ in range(3):
        db.check(False)
    ts = [db.check(False).stats["tier0_ms"] for _ in range(10)]
    print(f"keys {keys} mode {mode}: T0 {np.median(ts):.3f} ms", flush=True)
