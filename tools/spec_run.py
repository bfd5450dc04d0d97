"""C2 verdicts-only checks through the speculative path (profiling driver)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "jepsen-etcd-demo_amd"))
from lincheck import history as H  # noqa: E402
from lincheck.checker import Device, Packed  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4
h = H.synth(n_keys=1000, ops_per_key=1000, concurrency=10, seed=2)
pk = Packed(h)
dev = Device(0)
for _ in range(n):
    r = dev.check(pk, verdicts_only=True)
print("ok", r.stats["tier0_ms"], flush=True)
