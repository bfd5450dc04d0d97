"""C4 batch through the HBM tier once (profiling target).  With
LINCHECK_LIB_OVERRIDE=.../liblincheck_t3prof.so the kernel prints per-phase
cycles for the keys of its first blocks."""
import os, sys
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(root, "jepsen-etcd-demo_amd")]
from lincheck import history as H
from lincheck.checker import Device, Packed
budget = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 16
keys = int(sys.argv[2]) if len(sys.argv) > 2 else 256
probes = bool(int(sys.argv[3])) if len(sys.argv) > 3 else True
h = H.synth(n_keys=keys, ops_per_key=5000, concurrency=30, info_rate=0.02, seed=4)
db = Device(0, budget=budget, count_probes=probes).upload(Packed(h))
for i in range(2):
    st = db.check(False).stats
    print(f"iter {i}: kernel {st['kernel_ms']:.2f} ms t3 {st['tier3_ms']:.2f} ms probes {st['probes']} t3 {st['probes_t3']}",
          flush=True)
