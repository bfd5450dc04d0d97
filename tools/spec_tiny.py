"""One small register-tier check per setting, each under its own time limit
from the caller; prints the verdict agreement with the oracle."""
import os
import sys
import time

root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(root, "jepsen-etcd-demo_amd"), os.path.join(root, "oracle")]
import numpy as np  # noqa: E402

import cref  # noqa: E402
from lincheck import history as H  # noqa: E402
from lincheck.checker import Device, Packed  # noqa: E402

keys = int(sys.argv[1])
setting = sys.argv[2]
h = H.synth(n_keys=keys, ops_per_key=1000, concurrency=10, anomaly_rate=0.1, seed=5)
pk = Packed(h)
_, orc = cref.check_history(h.as_c(), budget=1 << 20, threads=8)
kw = {} if setting == "default" else {k: int(v, 0) for k, v in (kv.split("=") for kv in setting.split(","))}
dev = Device(0, **kw)
print("created", setting, flush=True)
t = time.perf_counter()
r = dev.check(pk, verdicts_only=True)
print(setting, keys, "t0_path", r.stats.get("t0_path"), "ms", round((time.perf_counter() - t) * 1e3, 2),
      "same", bool(np.array_equal(r.valid, orc["valid"]) and np.array_equal(r.fail_event, orc["fail_event"])),
      flush=True)
