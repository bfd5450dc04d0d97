"""C4 through the HBM tiers under one library build (LINCHECK_LIB_OVERRIDE
selects a variant): T3 time per check and a digest of the records, for A/B
runs of layered-tier variants.  usage: t3_ab.py [BUDGET] [REPS]"""
import hashlib
import os
import sys

root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(root, "jepsen-etcd-demo_amd")]
import numpy as np  # noqa: E402

from lincheck import history as H  # noqa: E402
from lincheck.checker import Device, Packed  # noqa: E402

budget = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 16
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
p = Packed(H.synth(n_keys=256, ops_per_key=5000, concurrency=30, info_rate=0.02, seed=4))
dev = Device(0, budget=budget)
db = dev.upload(p)
ts, ks = [], []
for _ in range(reps):
    r = db.check()
    ts.append(r.stats["tier3_ms"])
    ks.append(r.stats["kernel_ms"])
dig = hashlib.sha1(np.ascontiguousarray(r.valid).tobytes() + np.ascontiguousarray(r.fail_event).tobytes() +
                   np.ascontiguousarray(r.cause).tobytes()).hexdigest()[:12]
lib = os.path.basename(os.environ.get("LINCHECK_LIB_OVERRIDE", "liblincheck.so"))
print(f"{lib} budget {budget}: tier3 ms {np.round(ts, 2)} median {np.median(ts):.2f}  step ms median "
      f"{np.median(ks):.2f}  records {dig}", flush=True)
