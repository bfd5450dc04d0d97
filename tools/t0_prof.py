"""Cycles per event class in T0 (diagnostic build liblincheck_prof.so,
-DLC_T0_PROFILE): invoke, :ok with <= 6 / 7 / 8 / 9 / 10 ops pending."""
import os, sys, ctypes as C
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(root, "jepsen-etcd-demo_amd")]
import numpy as np
from lincheck import history as H
from lincheck import _native as N
from lincheck.checker import Device, Packed
h = H.synth(n_keys=1000, ops_per_key=1000, concurrency=10, seed=2)
pk = Packed(h)
st = Device(0).check(pk, verdicts_only=True).stats  # the bench's FAST path
buf = np.zeros(12, np.uint64)
N.lib().lc_debug_t0_prof(buf.ctypes.data_as(C.c_void_p))
cyc, cnt = buf[:6].astype(np.float64), buf[6:].astype(np.float64)
names = ["invoke", "ok<=6", "ok n=7", "ok n=8", "ok n=9", "ok n=10"]
tot = cyc.sum()
print("T0 ms (instrumented)", st["tier0_ms"])
for i, nm in enumerate(names):
    if cnt[i]:
        print("%-8s events/key %7.1f  cycles/event %7.0f  share %5.1f%%" %
              (nm, cnt[i] / pk.n_keys, cyc[i] / cnt[i], 100 * cyc[i] / tot))
print("cycles/key %.0f" % (tot / pk.n_keys))
