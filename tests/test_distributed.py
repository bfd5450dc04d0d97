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
    import torch.distributed as dist
    import cref
    from lincheck import history as H
    from lincheck import parallel as P
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    lo, hi = P.shard_range(n_keys, world, rank)
    block = -(-n_keys // world)
    h = H.synth(n_keys=hi - lo, ops_per_key=150, concurrency=6, anomaly_rate=0.3, seed=5, key_base=lo)
    keys, r = cref.check_history(h.as_c())
    # this rank's block exactly as lc_check_node lays it out (LC_REC_* words,
    # padded with 0 to the node's block), gathered in rank order
    node = P.gather_blocks(P.node_block(r["valid"], r["cause"], r["fail_event"], block))
    if rank == 0:
        np.save(out_path, node)
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gather_matches_single_process(tmp_path, world):
    """Each rank's shard as a block of LC_REC_* records (the library's node
    layout: include/lincheck.h), all-gathered over gloo, decoded by
    parallel.node_verdicts -- which the bench also uses on lc_check_node's
    gathered records -- equals a single-process check of every key."""
    import cref
    from lincheck import history as H
    n_keys = 37
    out = str(tmp_path / "gathered.npy")
    mp.spawn(_rank, args=(world, free_port(), n_keys, out), nprocs=world, join=True)
    node = np.load(out)
    block = -(-n_keys // world)
    sizes = [hi - lo for lo, hi in (parallel.shard_range(n_keys, world, r) for r in range(world))]
    assert node.size == block * world
    v, c, fe = parallel.node_verdicts(node, sizes, block)
    h = H.synth(n_keys=n_keys, ops_per_key=150, concurrency=6, anomaly_rate=0.3, seed=5)
    keys, r = cref.check_history(h.as_c())
    np.testing.assert_array_equal(v, r["valid"])
    np.testing.assert_array_equal(c, r["cause"])
    np.testing.assert_array_equal(fe, r["fail_event"])
    assert (v == 0).any()


def test_record_layout_is_the_header_s():
    """parallel.pack_records / unpack_records against include/lincheck.h's
    LC_REC_* macros, compiled."""
    import subprocess
    import tempfile
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    src = r"""
#include <stdio.h>
#include "lincheck.h"
int main(void) {
    unsigned long long r[3] = {%s};
    for (int i = 0; i < 3; ++i) printf("%%d %%d %%d\n", LC_REC_VALID(r[i]), LC_REC_CAUSE(r[i]), LC_REC_FAIL_EVENT(r[i]));
    return 0;
}"""
    v = np.array([1, 0, -1], np.int8); c = np.array([0, 1, 2], np.uint8); fe = np.array([-1, 17, 2**30], np.int32)
    rec = parallel.pack_records(v, c, fe)
    d = tempfile.mkdtemp()
    with open(os.path.join(d, "rec.c"), "w") as f:
        f.write(src % ", ".join(f"{int(x)}ull" for x in rec))
    subprocess.run(["gcc", "-I", os.path.join(root, "include"), "-o", os.path.join(d, "rec"),
                    os.path.join(d, "rec.c")], check=True)
    out = subprocess.run([os.path.join(d, "rec")], check=True, capture_output=True, text=True).stdout.split()
    got = np.array(out, np.int64).reshape(3, 3)
    np.testing.assert_array_equal(got[:, 0], v)
    np.testing.assert_array_equal(got[:, 1], c)
    np.testing.assert_array_equal(got[:, 2], fe)


def test_node_verdicts_refuses_records_in_padding():
    node = np.concatenate([parallel.node_block([1], [0], [-1], 3), parallel.node_block([0, 1, 1], [1, 0, 0], [5, -1, -1], 3)])
    v, _, fe = parallel.node_verdicts(node, [1, 3], 3)
    assert list(v) == [1, 0, 1, 1] and list(fe) == [-1, 5, -1, -1]
    with pytest.raises(ValueError):
        parallel.node_verdicts(node, [1, 2], 3)


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


def _mixed():
    from lincheck import history as H
    return H.History.concat([
        H.synth(n_keys=300, ops_per_key=300, concurrency=10, anomaly_rate=0.05, seed=7),
        H.synth(n_keys=100, ops_per_key=150, concurrency=6, anomaly_rate=0.1, seed=8, key_base=300),
        H.synth(n_keys=4, ops_per_key=200, concurrency=30, info_rate=0.02, seed=4, key_base=400)])


def _rank_cost(rank, world, port, out_path):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "jepsen-etcd-demo_amd"), os.path.join(root, "oracle")]
    import torch.distributed as dist
    import cref
    from lincheck import parallel as P
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    h = _mixed()
    keys, costs = P.key_costs(h, 1 << 16)
    shards = P.cost_shards(costs, world)
    block = max(len(s) for s in shards)
    sub = h.select_keys(keys[shards[rank]])
    k, r = cref.check_history(sub.as_c(), budget=1 << 16)
    assert list(k) == list(keys[shards[rank]])  # the shard's keys, in the caller's order
    node = P.gather_blocks(P.node_block(r["valid"], r["cause"], r["fail_event"], block))
    if rank == 0:
        np.save(out_path, node)
    dist.destroy_process_group()


def test_cost_sharded_mixed_batch(tmp_path):
    """VERDICT r5 next #5 / SURVEY E-1: a batch mixing C4-shaped keys
    (concurrency 30, crashed ops) into C5/C2-shaped ones, sharded by
    estimated cost (ops x concurrency x 2^crashed: parallel.key_costs,
    cost_shards) over a gloo world of 2; the node's records put back in the
    caller's key order equal one rank's check of the whole batch, and the
    ranks' estimated costs are within 10 % -- where the contiguous split
    leaves every C4-shaped key on one rank."""
    import cref
    h = _mixed()
    keys, costs = parallel.key_costs(h, 1 << 16)
    shards = parallel.cost_shards(costs, 2)
    loads = parallel.shard_costs(costs, shards)
    assert loads.max() <= 1.1 * loads.min()
    heavy = np.flatnonzero(costs > 10 * np.median(costs))
    assert len(heavy) >= 2 and set(heavy) <= {400, 401, 402, 403}  # C4-shaped keys are the heavy ones
    contig = [np.arange(*parallel.shard_range(len(costs), 2, r)) for r in range(2)]
    cl = parallel.shard_costs(costs, contig)
    assert cl.max() > 1.1 * cl.min()  # what cost sharding fixes
    out = str(tmp_path / "gathered.npy")
    mp.spawn(_rank_cost, args=(2, free_port(), out), nprocs=2, join=True)
    node = np.load(out)
    v, c, fe = parallel.node_key_order(node, shards, max(len(s) for s in shards))
    k, r = cref.check_history(h.as_c(), budget=1 << 16)
    assert list(k) == list(keys)
    np.testing.assert_array_equal(v, r["valid"])
    np.testing.assert_array_equal(c, r["cause"])
    np.testing.assert_array_equal(fe, r["fail_event"])
    assert (v == 0).any()


@pytest.mark.parametrize("world", [2, 3, 8])
def test_cost_shards_properties(world):
    rng = np.random.default_rng(world)
    for trial in range(20):
        costs = rng.pareto(1.5, size=int(rng.integers(1, 400))) + 0.01
        sh = parallel.cost_shards(costs, world)
        assert len(sh) == world
        allk = np.concatenate(sh)
        assert np.array_equal(np.sort(allk), np.arange(len(costs)))
        for s in sh:
            assert np.array_equal(s, np.sort(s))
        # no rank above the LPT bound: the fair share plus the largest key
        assert parallel.shard_costs(costs, sh).max() <= costs.sum() / world + costs.max() + 1e-9
    eq = parallel.cost_shards(np.ones(1001), world)
    assert all(parallel.contiguous(s) for s in eq) and max(map(len, eq)) - min(map(len, eq)) <= 1
