"""Offline fit of k_spec's TOP-walk cycles against the events each walk
covers (raw stamps from tools/spec_stamps.py ... OUT.npz, LC_SPEC_STAMPS
build): which event classes make the slow walks slow, and how well a
per-class cost model predicts them -- the weights the cost-balanced cuts use.
usage: spec_fit.py STAMPS.npz"""
import collections
import os
import sys

import numpy as np

root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(root, "jepsen-etcd-demo_amd")]
from lincheck import _native as N  # noqa: E402
from lincheck import history as H  # noqa: E402
from lincheck.checker import Packed  # noqa: E402

z = np.load(sys.argv[1])
b, keys, S = z["b"], int(z["keys"]), int(z["S"])
pk = Packed(H.synth(n_keys=keys, ops_per_key=1000, concurrency=10, seed=2))
nb = b.shape[0]
top = (b[:, :, 2] - b[:, :, 1]).astype(float)
info = b[:, :, 6]
hw = b[:, :, 8] & 0xFFFFFFFF
xcc = b[:, :, 8] >> 32
simd = (hw >> 4) & 3
cu = (hw >> 8) & 15
sh = (hw >> 12) & 1
se = (hw >> 13) & 7
place = list(zip(xcc.ravel(), se.ravel(), sh.ravel(), cu.ravel(), simd.ravel()))
cnt = collections.Counter(place)
per = np.array([cnt[p] for p in place]).reshape(xcc.shape).astype(float)


def walk_features(ev, c0, c1):
    """Event classes of events [c0, c1) of a key as the TOP walk sees them:
    op indices lowest-free from the cut's pending ops (slot order), the
    highest live index at each :ok, dirty :oks (an invoke since the last)."""
    ok = (ev & N.LC_EV_OK_BIT) != 0
    slot = (ev >> 24) & 0x7F
    pending = {}
    for j in range(c0):  # slots pending at the cut
        if ok[j]:
            pending.pop(int(slot[j]), None)
        else:
            pending[int(slot[j])] = True
    idx_of = {}
    live = 0
    for k, sl in enumerate(sorted(pending)):
        idx_of[sl] = k
        live |= 1 << k
    f = collections.Counter()
    dirty = True
    n = len(pending)
    for j in range(c0, c1):
        sl = int(slot[j])
        if not ok[j]:
            f["inv"] += 1
            if n < 6:
                i = (~live & (live + 1)).bit_length() - 1
            else:
                i = n
            idx_of[sl] = i
            live |= 1 << i
            n += 1
            dirty = True
        else:
            p = idx_of.pop(sl, 0)
            if n <= 6:
                t = live.bit_length()
                f[f"ok_T{min(max(t, 4), 6)}{'d' if dirty else 'c'}"] += 1
                live &= ~(1 << p)
            elif n <= 8:
                f["ok_78"] += 1
                last = n - 1
                for s2, i2 in list(idx_of.items()):
                    if i2 == last:
                        idx_of[s2] = p
                live = (1 << last) - 1
            else:
                f["ok_910"] += 1
                last = n - 1
                for s2, i2 in list(idx_of.items()):
                    if i2 == last:
                        idx_of[s2] = p
                live = (1 << last) - 1
            dirty = n > 6  # the lane phase closes its set; the dense phase hands on an exact one
            n -= 1
    return f


names = ["inv", "ok_T4c", "ok_T4d", "ok_T5c", "ok_T5d", "ok_T6c", "ok_T6d", "ok_78", "ok_910"]
rows = []
keyid = b[:, 0, 9]
for bi in range(nb):
    ev = pk.events(int(keyid[bi]))
    for w in range(S):
        c0, c1 = int(info[bi, w] & 0xFFFFFFFF), int(info[bi, w] >> 32)
        f = walk_features(ev, c0, c1)
        rows.append([f.get(k, 0) for k in names])
F = np.array(rows, float)
y = top.ravel()
pw = per.ravel()
X = np.column_stack([F, F.sum(1) * pw])
coef, *_ = np.linalg.lstsq(X, y, rcond=None)
pred = X @ coef
r2 = 1 - ((y - pred) ** 2).sum() / ((y - y.mean()) ** 2).sum()
print("fit (cycles per event of each class; last: per event per co-resident wave):")
for k, c in zip(names + ["ev_x_waves"], coef):
    print(f"  {k:>10} {c:9.1f}")
print(f"R^2 {r2:.3f}  median walk {np.median(y):.0f}  max {y.max():.0f}  predicted max {pred.max():.0f}")
o = np.argsort(-y)[:10]
print("slowest walks: cycles, predicted, events, " + " ".join(names))
for j in o:
    print(f"  {y[j]:8.0f} {pred[j]:8.0f} {F[j].sum():5.0f} " + " ".join(f"{int(x):4d}" for x in F[j]))
# per key: total predicted cost (what cost-balanced cuts could at best equalise)
kc = pred.reshape(nb, S).sum(1)
print(f"per-key predicted total / {S}: median {np.median(kc) / S:.0f} max {kc.max() / S:.0f}")
res = y - pred
print(f"residual std {res.std():.0f}; slowest-walk residuals {np.round(res[o]).astype(int).tolist()}")
# where the unexplained time sits: by segment, XCC, block position, CU load
R = res.reshape(nb, S)
print("residual by segment:", [int(np.mean(R[:, w])) for w in range(S)])
print("residual by XCC:", {int(x): int(np.mean(res[xcc.ravel() == x])) for x in sorted(set(xcc.ravel().tolist()))})
dec = np.repeat(np.arange(nb) * 10 // nb, S)
print("residual by block-index decile:", [int(np.mean(res[dec == d])) for d in range(10)])
cus = collections.Counter(zip(xcc.ravel(), se.ravel(), sh.ravel(), cu.ravel()))
cuw = np.array([cus[p] for p in zip(xcc.ravel(), se.ravel(), sh.ravel(), cu.ravel())])
print("residual by waves on the CU:", {int(k): int(np.mean(res[cuw == k])) for k in sorted(set(cuw.tolist()))})
# blocks of one CU: does the whole CU run slow?
cu_id = [hash(p) for p in zip(xcc.ravel(), se.ravel(), sh.ravel(), cu.ravel())]
by_cu = collections.defaultdict(list)
for i, c in enumerate(cu_id):
    by_cu[c].append(res[i])
cm = np.array([np.mean(v) for v in by_cu.values()])
print(f"per-CU mean residual: std {cm.std():.0f}  (walk residual std {res.std():.0f}); "
      f"fraction of variance between CUs {cm.var() / res.var():.2f}")
blk = R.mean(1)
print(f"per-block mean residual: std {blk.std():.0f}; fraction of variance between blocks {blk.var() / res.var():.2f}")
