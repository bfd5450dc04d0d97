"""Runs T0 on the C2 batch repeatedly (profiling target); prints per-iteration T0 time."""
import os, sys, time
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(root, "jepsen-etcd-demo_amd")]
import numpy as np
from lincheck import history as H
from lincheck.checker import Device, Packed
mode = int(sys.argv[1]) if len(sys.argv) > 1 else 0
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 4
h = H.synth(n_keys=1000, ops_per_key=1000, concurrency=10, seed=2)
pk = Packed(h)
db = Device(0, debug_mode=mode).upload(pk)
ts = []
t0 = time.time()
for _ in range(iters):
    ts.append(db.check(False).stats["tier0_ms"])
ts = np.array(ts)
print(f"iters {iters} wall {time.time()-t0:.2f}s  T0 ms first {ts[:5].round(3)} last {ts[-5:].round(3)} min {ts.min():.3f} median {np.median(ts):.3f}")
