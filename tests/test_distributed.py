"""Multi-rank path on CPU (gloo, world_size 2): each rank checks its own key
shard and the verdict records are all-gathered, as bench.py does over RCCL.
The merged verdicts must equal a single-process check of all keys."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from lincheck import parallel


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank(rank, world, port, n_keys, out_path):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "jepsen-etcd-demo_amd"), os.path.join(root, "oracle")]
    import torch
    import torch.distributed as dist
    import cref
    from lincheck import history as H
    from lincheck import parallel as P
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    lo, hi = P.shard_range(n_keys, world, rank)
    h = H.synth(n_keys=hi - lo, ops_per_key=150, concurrency=6, anomaly_rate=0.3, seed=5, key_base=lo)
    keys, r = cref.check_history(h.as_c())
    rec = P.pack_records(r["valid"], r["cause"], r["fail_event"])
    ks, rs = P.gather_records(torch.from_numpy(keys.astype(np.int64)), torch.from_numpy(rec))
    if rank == 0:
        np.save(out_path, np.stack([ks, rs]))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_gather_matches_single_process(tmp_path, world):
    import cref
    from lincheck import history as H
    n_keys = 37
    out = str(tmp_path / "gathered.npy")
    mp.spawn(_rank, args=(world, free_port(), n_keys, out), nprocs=world, join=True)
    ks, rs = np.load(out)
    h = H.synth(n_keys=n_keys, ops_per_key=150, concurrency=6, anomaly_rate=0.3, seed=5)
    keys, r = cref.check_history(h.as_c())
    assert list(ks) == list(keys)
    v, c, fe = parallel.unpack_records(rs)
    np.testing.assert_array_equal(v, r["valid"])
    np.testing.assert_array_equal(c, r["cause"])
    np.testing.assert_array_equal(fe, r["fail_event"])
    assert (v == 0).any()


def test_shards_cover_keys():
    for n in (0, 1, 7, 1000):
        for w in (1, 2, 3, 8):
            rngs = [parallel.shard_range(n, w, r) for r in range(w)]
            assert rngs[0][0] == 0 and rngs[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(rngs, rngs[1:]))
            assert max(h - l for l, h in rngs) - min(h - l for l, h in rngs) <= 1


def test_lpt_balances():
    costs = [100, 1, 1, 1, 50, 50, 3, 90]
    sh = parallel.lpt_shards(costs, 3)
    assert sorted(np.concatenate(sh).tolist()) == list(range(len(costs)))
    loads = [sum(costs[i] for i in s) for s in sh]
    assert max(loads) <= 103


def test_record_round_trip():
    v = np.array([1, 0, -1], np.int8); c = np.array([0, 1, 2], np.uint8); fe = np.array([-1, 17, 2**30], np.int32)
    vv, cc, ff = parallel.unpack_records(parallel.pack_records(v, c, fe))
    assert (vv == v).all() and (cc == c).all() and (ff == fe).all()
