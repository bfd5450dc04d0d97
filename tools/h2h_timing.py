"""Breakdown of lc_check_batch (host SoA -> host verdicts) on the C2 batch:
LC_TIMING=1 makes the library print validate / upload / check times."""
import os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "jepsen-etcd-demo_amd"))
os.environ["LC_TIMING"] = "1"
from lincheck import history as H
from lincheck.checker import Device, Packed
h = H.synth(n_keys=1000, ops_per_key=1000, concurrency=10, seed=2)
pk = Packed(h)
dev = Device(0)
for i in range(6):
    t = time.perf_counter()
    r = dev.check(pk, verdicts_only=True)
    w = (time.perf_counter() - t) * 1e3
    print(f"call {i}: wall {w:.3f} ms, total_ms {r.stats['total_ms']:.3f}, kernel_ms {r.stats['kernel_ms']:.3f}", flush=True)
