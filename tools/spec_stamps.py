"""Phase stamps of the speculative-segment kernel (diagnostic build:
make variant NAME=specst VFLAGS=-DLC_SPEC_STAMPS, then
LINCHECK_LIB_OVERRIDE=.../liblincheck_specst.so python tools/spec_stamps.py)."""
import ctypes as C
import os
import sys

import numpy as np

root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(root, "jepsen-etcd-demo_amd")]
from lincheck import _native as N  # noqa: E402
from lincheck import history as H  # noqa: E402
from lincheck.checker import Device, Packed  # noqa: E402

keys = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
S = int(sys.argv[2]) if len(sys.argv) > 2 else 4         # segments per key (lc_opts.spec_segs)
flags = int(sys.argv[3], 0) if len(sys.argv) > 3 else 0  # lc_opts.path_flags (e.g. 0x100: even cuts)
# SPEC_CFG=C5: the C5 shape (5 % anomalous keys, seed 5); default C2
h = H.synth(**dict(H.CONFIGS[os.environ.get("SPEC_CFG", "C2")], n_keys=keys))
pk = Packed(h)
dev = Device(0, spec_segs=S, path_flags=flags)
for _ in range(10):
    st = dev.check(pk, verdicts_only=True).stats
nb = min(keys, 4096)
buf = np.zeros(nb * 8 * 12, np.uint64)
N.lib().lc_debug_spec_stamps(buf.ctypes.data_as(C.c_void_p), nb)
b = buf.reshape(nb, 8, 12).astype(np.int64)[:, :S, :]
if len(sys.argv) > 4:  # raw stamps for offline fits (the keys regenerate from the seed)
    np.savez(sys.argv[4], b=b, keys=keys, S=S, flags=flags)
t0 = b[:, :, 0].min()
print("T0 ms", st["tier0_ms"], "blocks", nb, "segments", S)
start = b[:, :, 0] - t0
cut = b[:, :, 1] - b[:, :, 0]
top = b[:, :, 2] - b[:, :, 1]
bar1 = b[:, :, 3] - b[:, :, 2]
ver = b[:, :, 4] - b[:, :, 3]
bar2 = b[:, :, 5] - b[:, :, 4]
end = b[:, :, 5] - t0
info = b[:, :, 6]
seg_len = (info >> 32) - (info & 0xFFFFFFFF)
v = b[:, 1:, 7]


def q(x):
    return "median %8.0f p90 %8.0f max %8.0f" % (np.median(x), np.percentile(x, 90), x.max())


print("start offset cycles  ", q(start))
print("cut computation      ", q(cut))
print("TOP walk             ", q(top))
print("TOP cycles per event ", q(top / np.maximum(seg_len, 1)))
print("wait at barrier 1    ", q(bar1))
print("verify               ", q(ver[:, 1:]))
print("wait at barrier 2    ", q(bar2))
print("block end (from t0)  ", q(end.max(1)))
print("verify events        ", q(v & 0xFFFFFFFF))
print("verify outcomes      ", {int(k): int(c) for k, c in zip(*np.unique(v >> 32, return_counts=True))})
print("segment lengths      ", q(seg_len))

# co-residency: waves per SIMD, and what the slow TOP walks have in common
import collections
hw = b[:, :, 8] & 0xFFFFFFFF
xcc = b[:, :, 8] >> 32
simd = (hw >> 4) & 3; cu = (hw >> 8) & 15; sh = (hw >> 12) & 1; se = (hw >> 13) & 7
place = list(zip(xcc.ravel(), se.ravel(), sh.ravel(), cu.ravel(), simd.ravel()))
cnt = collections.Counter(place)
per = np.array([cnt[p] for p in place]).reshape(xcc.shape)
cus = collections.Counter(zip(xcc.ravel(), se.ravel(), sh.ravel(), cu.ravel()))
print("distinct SIMDs", len(cnt), "waves per SIMD", dict(collections.Counter(cnt.values())),
      "distinct CUs", len(cus), "waves per CU", dict(collections.Counter(cus.values())))
tw = top.ravel().astype(float)
keyid = b[:, 0, 9]
dense = np.zeros(b.shape[:2]); deep = np.zeros(b.shape[:2])
for bi in range(nb):
    ev = pk.events(int(keyid[bi]))
    okb = (ev & N.LC_EV_OK_BIT) != 0
    pend = np.cumsum(np.where(okb, -1, 1))
    for w in range(S):
        c0, c1 = int(info[bi, w] & 0xFFFFFFFF), int(info[bi, w] >> 32)
        m = okb[c0:c1]; pn = pend[c0:c1] + 1
        dense[bi, w] = ((pn >= 7) & m).sum(); deep[bi, w] = ((pn >= 9) & m).sum()
for k in (1, 2, 3, 4):
    m = per.ravel() == k
    if m.any():
        print("waves on SIMD %d: n %5d  TOP cycles/event median %.0f" % (k, m.sum(), np.median((top / np.maximum(seg_len, 1)).ravel()[m])))
X = np.column_stack([seg_len.ravel(), dense.ravel(), deep.ravel(), per.ravel() * seg_len.ravel()]).astype(float)
coef, *_ = np.linalg.lstsq(X, tw, rcond=None)
print("fit TOP cycles: per event %.0f, per dense :ok %.0f, per 9-10 :ok %.0f, per event x waves/SIMD %.0f" % tuple(coef))
o = np.argsort(-tw)[:8]
print("slowest TOP walks: cycles, events, dense oks, 9-10 oks, waves on its SIMD")
for j in o:
    print("  %8d %5d %4d %4d %d" % (tw[j], seg_len.ravel()[j], dense.ravel()[j], deep.ravel()[j], per.ravel()[j]))

# per SIMD: the sum of its waves' work against its slowest TOP walk
simd_of = {}
for idx, pl in enumerate(place):
    simd_of.setdefault(pl, []).append(idx)
wl = seg_len.ravel().astype(float) + dense.ravel() * 0.35 + deep.ravel() * 22.0
sums = np.array([wl[v].sum() for v in simd_of.values()])
mx = np.array([tw[v].max() for v in simd_of.values()])
print("per-SIMD weighted work: median %.0f p90 %.0f max %.0f; corr with its slowest TOP %.3f"
      % (np.median(sums), np.percentile(sums, 90), sums.max(), np.corrcoef(sums, mx)[0, 1]))
xr = xcc.ravel()
for x in sorted(set(xr.tolist())):
    m = xr == x
    print("xcc %d: TOP cycles/event median %.0f p90 %.0f" % (x, np.median((tw / np.maximum(seg_len.ravel(), 1))[m]),
                                                            np.percentile((tw / np.maximum(seg_len.ravel(), 1))[m], 90)))

# the launch's tail: the slowest blocks, segment by segment (C5: the invalid
# keys' verifying runs)
ends = end.max(1)
print("slowest blocks: key, block end; per segment: TOP cycles / events, verify cycles / events / outcome")
for bi in np.argsort(-ends)[:6]:
    segs = []
    for w in range(S):
        vv = int(b[bi, w, 7]) if w else 0
        segs.append("%d/%d v%d/%d/%d" % (top[bi, w], seg_len[bi, w], ver[bi, w] if w else 0, vv & 0xFFFFFFFF,
                                          vv >> 32))
    print("  key %6d end %8d  %s" % (keyid[bi], ends[bi], "  ".join(segs)))
