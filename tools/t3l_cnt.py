"""C4 through the layered HBM tier with the LC_T3L_CNT variant
(LINCHECK_LIB_OVERRIDE=.../liblincheck_t3lcnt.so): per-key phase cycles and
step counts from the final-config words.  Diagnostic only."""
import os, sys
import numpy as np
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(root, "jepsen-etcd-demo_amd")]
from lincheck import history as H
from lincheck.checker import Device, Packed
budget = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 16
keys = int(sys.argv[2]) if len(sys.argv) > 2 else 256
h = H.synth(n_keys=keys, ops_per_key=5000, concurrency=30, info_rate=0.02, seed=4)
p = Packed(h)
dev = Device(0, budget=budget)
for it in range(2):
    r = dev.check(p)
    print(f"iter {it}: kernel {r.stats['kernel_ms']:.2f} ms t3 {r.stats['tier3_ms']:.2f} ms", flush=True)
qa = r.final.reshape(len(p.keys), -1).astype(np.int64)
q = qa[:, :10]
# whole-table steps: insert cycles, scan cycles, I passes, S' passes, pairs + S entries per I pass (thread 0)
ws = qa[:, 10:16]
names = ["between", "okhead", "inserts", "scans", "fast", "slowcyc", "oks", "entries", "redo|slow<<20", "total"]
order = np.argsort(-q[:, 9])
for i in order[:6]:
    d = dict(zip(names, q[i].tolist()))
    d["slow"] = d["redo|slow<<20"] >> 20
    d["redo"] = d["redo|slow<<20"] & 0xFFFFF
    print(i, d, "cyc/step", d["total"] // max(1, d["fast"] + d["slow"]))
    w = ws[i]
    print("   whole-table: inserts %d cyc, scans %d cyc (%.1f%% / %.1f%% of the key), I passes %d, S' passes %d, "
          "inputs per I pass %.0f" % (w[0], w[1], 100 * w[0] / d["total"], 100 * w[1] / d["total"], w[2], w[3],
                                      w[5] / max(1, w[2])))
tot = q.sum(0)
print("sums", dict(zip(names, tot.tolist())))
