"""A/B of T0 builds on one box: resident C2 steps (lc_check_node_device,
asynchronous) with the library named in argv[1]; prints T0 ms per launch."""
import os, sys
os.environ["LINCHECK_LIB_OVERRIDE"] = os.path.abspath(sys.argv[1])
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(root, "jepsen-etcd-demo_amd")]
import numpy as np
from lincheck import history as H
from lincheck.checker import Device, Packed
keys, ops = (int(sys.argv[2]), int(sys.argv[3])) if len(sys.argv) > 3 else (1000, 1000)
pk = Packed(H.synth(n_keys=keys, ops_per_key=ops, concurrency=10, seed=2))
dev = Device(0)
db = dev.upload(pk)
out = []
for rep in range(5):
    for _ in range(30):
        db.check_node(pk.n_keys, asynchronous=True)
    n, span = dev.wait()
    out.append(span / n)
print(f"{os.path.basename(sys.argv[1])}: T0 ms per launch {np.round(out, 4)} median {np.median(out):.4f}", flush=True)
