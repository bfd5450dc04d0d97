"""Resident C2 steps (lc_check_node_device, asynchronous) under a list of
lc_opts path settings, one line each: the span per step from lc_wait (HIP
events).  A setting is comma-separated key=value pairs of Device() options
(path_flags=<int>, spec_segs=<n>, seg_len=<n>); verdicts are checked against
the first setting's."""
import os, sys
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(root, "jepsen-etcd-demo_amd")]
import numpy as np
from lincheck import history as H
from lincheck.checker import Device, Packed
keys, ops = int(os.environ.get("SW_KEYS", 1000)), int(os.environ.get("SW_OPS", 1000))
pk = Packed(H.synth(n_keys=keys, ops_per_key=ops, concurrency=int(os.environ.get("SW_CONC", 10)), seed=2,
                    mean_think=float(os.environ.get("SW_THINK", 1.0))))
ref = None
for setting in sys.argv[1:]:
    kw = {k: int(v, 0) for k, v in (kv.split("=") for kv in filter(None, setting.split(",")))}
    dev = Device(0, **kw)
    db = dev.upload(pk)
    out = []
    for rep in range(4):
        for _ in range(20):
            db.check_node(pk.n_keys, asynchronous=True)
        n, span = dev.wait()
        out.append(span / n)
    rec = dev.node_records(pk.n_keys)
    ref = rec if ref is None else ref
    print(f"{setting or 'default':>28}: ms/step {np.round(out, 4)} median {np.median(out):.4f} same {np.array_equal(rec, ref)}",
          flush=True)
