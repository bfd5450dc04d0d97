"""Diagnostic: device T0 vs the C oracle on a C2-shaped batch; prints the
mismatching keys with the pending count at the device's failing event."""
import sys, os
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(root, "jepsen-etcd-demo_amd"), os.path.join(root, "oracle")]
import numpy as np
from lincheck import history as H
from lincheck.checker import Device, Packed
import cref

h = H.synth(n_keys=300, ops_per_key=1000, concurrency=10, seed=2)
pk = Packed(h)
res = Device(0).check(pk)
keys, orc = cref.check_history(h.as_c(), threads=8)
bad = np.nonzero((res.valid != orc["valid"]) | (res.fail_event != orc["fail_event"]))[0]
print(os.environ.get("LINCHECK_LIB_OVERRIDE", "default"), "mismatches", len(bad), "deep", res.stats["deep_keys"])
for i in bad[:12]:
    ev = pk.events(i); n = 0; hist = []
    fe = int(res.fail_event[i])
    for j, w in enumerate(ev[:fe + 1] if fe >= 0 else ev):
        if w & 0x80000000:
            hist.append(n); n -= 1
        else:
            n += 1
    print(f" key {i}: dev {res.valid[i]} fe {fe} | oracle {orc['valid'][i]} {orc['fail_event'][i]} | n at fail {hist[-1] if hist else None} max n so far {max(hist) if hist else None} last ns {hist[-8:]}")
