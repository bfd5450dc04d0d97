"""Breakdown of lc_check_node (the bench's D-1 step) on the C2 batch:
LC_TIMING=1 makes the library print prepare / upload / enqueue / wait times."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "jepsen-etcd-demo_amd"))
os.environ["LC_TIMING"] = "1"
from lincheck import history as H  # noqa: E402
from lincheck.checker import Device, Packed  # noqa: E402

h = H.synth(n_keys=1000, ops_per_key=1000, concurrency=10, seed=2)
pk = Packed(h)
dev = Device(0)
for i in range(8):
    t = time.perf_counter()
    _, st = dev.check_node(pk, pk.n_keys)
    print(f"call {i}: wall {(time.perf_counter() - t) * 1e3:.3f} ms", file=sys.stderr, flush=True)
