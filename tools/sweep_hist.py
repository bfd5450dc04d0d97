"""Histogram of closure sweeps per :ok in T0's lane tier (diagnostic build
liblincheck_sweeps.so, -DLC_T0_COUNT_SWEEPS)."""
import os, sys, ctypes as C
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(root, "jepsen-etcd-demo_amd")]
import numpy as np
from lincheck import history as H
from lincheck import _native as N
from lincheck.checker import Device, Packed
h = H.synth(n_keys=1000, ops_per_key=1000, concurrency=10, seed=2)
pk = Packed(h)
Device(0).check(pk)
buf = np.zeros(64, np.uint64)
N.lib().lc_debug_sweep_hist(buf.ctypes.data_as(C.c_void_p))
hist = buf.reshape(8, 8)
tot = hist.sum()
print("ok_lane events", tot)
for nc in range(8):
    if hist[nc].sum():
        print("nc=%d: %7d events (%.1f%%), sweeps run:" % (nc, hist[nc].sum(), 100 * hist[nc].sum() / tot),
              " ".join("%d:%d" % (s, hist[nc, s]) for s in range(8) if hist[nc, s]))
avg = sum(hist[nc, s] * s for nc in range(8) for s in range(8)) / tot
print("mean sweeps per ok: %.2f" % avg)
