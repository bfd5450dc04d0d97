"""Per-block clock stamps of T0 (diagnostic build liblincheck_stamps.so)."""
import os, sys, ctypes as C, collections
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(root, "jepsen-etcd-demo_amd")]
import numpy as np
from lincheck import history as H
from lincheck import _native as N
from lincheck.checker import Device, Packed
keys = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
h = H.synth(n_keys=keys, ops_per_key=1000, concurrency=10, seed=2)
pk = Packed(h)
db = Device(0).upload(pk)
for _ in range(20):
    st = db.check(False).stats
nb = min(keys, 4096)
buf = np.zeros(nb * 6, np.uint64)
rc = N.lib().lc_debug_t0_stamps(buf.ctypes.data_as(C.c_void_p), nb)
b = buf.reshape(nb, 6).astype(np.int64)
cyc = b[:, 1] - b[:, 0]; rt = b[:, 3] - b[:, 2]
print("rc", rc, "T0 ms", st["tier0_ms"])
print("per-block cycles: min %d median %d max %d" % (cyc.min(), np.median(cyc), cyc.max()))
print("per-block realtime ticks (100MHz): min %d median %d max %d" % (rt.min(), np.median(rt), rt.max()))
print("clock GHz (cycles/realtime*0.1):", np.median(cyc / np.maximum(rt, 1)) * 0.1)
start_rt = b[:, 2] - b[:, 2].min(); end_rt = b[:, 3] - b[:, 2].min()
print("start spread us: max %.1f ; end max us %.1f" % (start_rt.max() / 100, end_rt.max() / 100))
hw = b[:, 4] & 0xFFFFFFFF; xcc = b[:, 5] & 0xFFFFFFFF; nk = b[:, 5] >> 32
simd = (hw >> 4) & 3; cu = (hw >> 8) & 15; sh = (hw >> 12) & 1; se = (hw >> 13) & 7
place = collections.Counter(zip(xcc, se, sh, cu, simd))
print("distinct SIMDs", len(place), "max blocks on one SIMD", max(place.values()), "keys per block max", nk.max())
cuc = collections.Counter(zip(xcc, se, sh, cu))
print("distinct CUs", len(cuc), "max blocks per CU", max(cuc.values()))

# per-key critical path vs the key's shape (one key per block when keys <= grid)
if nk.max() == 1:
    kid = b[:, 4] >> 32
    width = np.ctypeslib.as_array(pk.view.key_width, shape=(pk.n_keys,))
    nev = np.diff(pk.ev_off.astype(np.int64))
    hi = np.zeros(pk.n_keys, np.int64)   # :ok events with >= 7 ops pending
    byn = np.zeros((pk.n_keys, 11), np.int64)  # :ok events by ops pending
    for i in range(pk.n_keys):
        ev = pk.events(i)
        okb = (ev & N.LC_EV_OK_BIT) != 0
        pend = np.cumsum(np.where(okb, -1, 1))  # pending after each event
        hi[i] = int(((pend + 1 >= 7) & okb).sum())
        byn[i] = np.bincount(np.minimum(pend[okb] + 1, 10), minlength=11)
    c = cyc.astype(np.float64)
    w = width[kid]; hk = hi[kid]; ne = nev[kid]
    print("cycles per event: median %.0f max %.0f" % (np.median(c / ne), (c / ne).max()))
    for wv in sorted(set(w.tolist())):
        m = w == wv
        print("width %2d: keys %4d  cycles median %9.0f max %9.0f  ok>=7 pending median %d" %
              (wv, m.sum(), np.median(c[m]), c[m].max(), np.median(hk[m])))
    order = np.argsort(-c)[:10]
    print("slowest keys: cycles / width / ok>=7 / events / oks at n=7,8,9,10")
    for j in order:
        print("  %9d %3d %5d %6d   %s" % (c[j], w[j], hk[j], ne[j], byn[kid[j], 7:11].tolist()))
    # least squares: cycles ~ a*invokes + b*ok(<=6) + c7*ok7 + c8*ok8 + c9*ok9 + c10*ok10
    nb = byn[kid]
    X = np.column_stack([ne - nb.sum(1), nb[:, :7].sum(1), nb[:, 7], nb[:, 8], nb[:, 9], nb[:, 10]]).astype(np.float64)
    coef, *_ = np.linalg.lstsq(X, c, rcond=None)
    print("fit cycles per event: invoke %.0f ok<=6 %.0f ok7 %.0f ok8 %.0f ok9 %.0f ok10 %.0f" % tuple(coef))
    print("corr(cycles, ok>=7 pending) = %.3f" % np.corrcoef(c, hk)[0, 1])
