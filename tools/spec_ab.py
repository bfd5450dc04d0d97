"""A/B of register-tier path options on one batch: resident node steps
(lc_check_node_device, asynchronous; span per step from lc_wait) and the
bench's pipelined step (lc_check_node_async), per lc_opts setting, records
checked equal across settings.
usage: spec_ab.py CONFIG KEYS OPS SETTING...   (SETTING: k=v,k=v Device options,
e.g. path_flags=0x100 or spec_segs=8; "default" for none)"""
import os
import sys
import time

root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(root, "jepsen-etcd-demo_amd")]
import numpy as np  # noqa: E402

from lincheck import history as H  # noqa: E402
from lincheck.checker import Device, Packed, PinnedRecords  # noqa: E402

cfg, keys, ops = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
shape = dict(C2=dict(concurrency=10, seed=2), C5=dict(concurrency=10, anomaly_rate=0.05, seed=5),
             C3=dict(concurrency=10, seed=3))[cfg]
if os.environ.get("SEED"):  # another instance of the same shape
    shape = dict(shape, seed=int(os.environ["SEED"]))
pk = Packed(H.synth(n_keys=keys, ops_per_key=ops, **shape))
K = pk.n_keys
ref = None
for setting in sys.argv[4:]:
    kw = {} if setting == "default" else {k: int(v, 0) for k, v in (kv.split("=") for kv in setting.split(","))}
    if "spec_ck" in kw:  # (ck1 + 1) | (ck2 + 1) << 16, as lc_opts.spec_ck
        kw["spec_ck"] = ((kw["spec_ck"] & 0xFFFF) - 1, (kw["spec_ck"] >> 16) - 1)
    dev = Device(0, **kw)
    db = dev.upload(pk)
    for _ in range(10):
        db.check_node(K, asynchronous=True)
    dev.wait()
    res = []
    for rep in range(5):
        for _ in range(40):
            db.check_node(K, asynchronous=True)
        n, span = dev.wait()
        res.append(span / max(n, 1))
    rec = dev.node_records(K)
    del db
    bufs = [PinnedRecords(K) for _ in range(2)]
    for i in range(10):
        dev.check_node_async(pk, K, bufs[i & 1])
    dev.wait()
    t = time.perf_counter()
    for i in range(100):
        dev.check_node_async(pk, K, bufs[i & 1])
    dev.wait()
    pipe = (time.perf_counter() - t) / 100 * 1e3
    same_pipe = bool(np.array_equal(np.asarray(bufs[1]), rec))
    ref = rec if ref is None else ref
    print(f"{cfg} {K}x{ops} {setting:>28}: resident ms/step {np.round(res, 4)} median {np.median(res):.4f}  "
          f"pipelined {pipe:.4f} ms  same {np.array_equal(rec, ref)} {same_pipe}", flush=True)
    del dev
