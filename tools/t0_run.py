"""Runs T0 on the C2 batch a few times (profiling target)."""
import os, sys
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(root, "jepsen-etcd-demo_amd")]
from lincheck import history as H
from lincheck.checker import Device, Packed
mode = int(sys.argv[1]) if len(sys.argv) > 1 else 0
h = H.synth(n_keys=1000, ops_per_key=1000, concurrency=10, seed=2)
pk = Packed(h)
db = Device(0, debug_mode=mode).upload(pk)
for _ in range(4):
    st = db.check(False).stats
print("T0 ms", st["tier0_ms"])
