"""Multi-device contexts, node-wide verdict records and batches T0 validates.

* independent/checker's pmap over a node's
  GPUs (etcdemo.clj:115).  A context over several devices checks contiguous
  key shards at once; on this one-GPU box the shards are logical (devices
  [0, 0] and [0, 0, 0]: one stream and scratch per shard on the same card),
  and every result array must equal the one-shard check bit for bit.
* lc_check_node: a rank's shard -> verdict records all-gathered over the
  node.  One rank here, with and without a (one-rank) RCCL communicator:
  the decoded records must equal lc_check_batch's verdicts.
* A batch whose keys all fit the register tier is validated by T0 while it
  walks the events: each malformation is refused (LC_E_INVALID naming the
  key) on the host-to-host, resident and asynchronous paths, and the
  context keeps working.
"""
import ctypes as C
import os

import numpy as np
import pytest

import cref
from helpers import device_vs_oracle
from lincheck import _native as N
from lincheck import history as H
from lincheck import parallel as P
from lincheck.checker import Device, Packed, comm_id

pytestmark = pytest.mark.gpu

SHAPES = {
    # register tier only (T0-validated batches)
    "c5": dict(n_keys=300, ops_per_key=400, concurrency=10, anomaly_rate=0.1, seed=71),
    # keys leave T0 (host-validated; T1-T3 run)
    "crashed": dict(n_keys=24, ops_per_key=500, concurrency=14, info_rate=0.01, anomaly_rate=0.2, seed=72),
}


def _same(a, b, max_final=10):
    for f in ("valid", "fail_event", "cause", "peak", "n_final"):
        np.testing.assert_array_equal(getattr(a, f), getattr(b, f), err_msg=f)
    for i in range(len(a.valid)):
        n = int(a.n_final[i])
        if n < max_final:  # the whole final set: equal as a set (hash tiers append in any order)
            sa = sorted(map(tuple, a.final[i, :n].tolist()))
            sb = sorted(map(tuple, b.final[i, :n].tolist()))
            assert sa == sb, f"final configs of key {i}"


@pytest.mark.parametrize("shape", sorted(SHAPES))
@pytest.mark.parametrize("devices", [[0, 0], [0, 0, 0]])
def test_logical_shards_bit_exact(shape, devices):
    h = H.synth(**SHAPES[shape])
    pk = Packed(h)
    one = Device(0).check(pk)
    multi = Device(0, devices=devices)
    _same(multi.check(pk), one)
    _same(multi.upload(pk).check(), one)  # resident shards, host results
    _, orc = cref.check_history(h.as_c(), budget=1 << 20, threads=8)
    np.testing.assert_array_equal(one.valid, orc["valid"])
    np.testing.assert_array_equal(one.fail_event, orc["fail_event"])


def test_logical_shards_more_than_keys():
    """Three shards over two keys: a shard with no keys is a no-op."""
    h = H.synth(n_keys=2, ops_per_key=300, concurrency=8, anomaly_rate=0.5, seed=73)
    dev = Device(0, devices=[0, 0, 0])
    device_vs_oracle(h, dev)


def _decode(rec, K):
    v, c, fe = P.unpack_records(rec.astype(np.int64))
    return v[:K], c[:K], fe[:K]


@pytest.mark.parametrize("shape", sorted(SHAPES))
@pytest.mark.parametrize("rccl", [False, True])
def test_node_records_one_rank(shape, rccl):
    h = H.synth(**SHAPES[shape])
    pk = Packed(h)
    K = pk.n_keys
    ref = Device(0).check(pk)
    dev = Device(0, comm=(0, 1, comm_id()) if rccl else None)
    block = K + 7  # padded block: the padding records are 0
    rec, _ = dev.check_node(pk, block)
    assert rec.size == block and not rec[K:].any()
    v, c, fe = _decode(rec, K)
    np.testing.assert_array_equal(v, ref.valid)
    np.testing.assert_array_equal(c, ref.cause)
    np.testing.assert_array_equal(fe, ref.fail_event)
    # resident shard: synchronous, then asynchronous steps + lc_wait
    db = dev.upload(pk)
    db.check_node(block)
    np.testing.assert_array_equal(dev.node_records(block), rec)
    for _ in range(3):
        db.check_node(block, asynchronous=True)
    dev.wait()
    np.testing.assert_array_equal(dev.node_records(block), rec)


def test_node_block_too_small():
    pk = Packed(H.synth(n_keys=10, ops_per_key=50, concurrency=4, seed=74))
    with pytest.raises(N.LincheckError) as ei:
        Device(0).check_node(pk, 9)
    assert ei.value.code == -1


def _batch_copy(pk):
    """Writable copies of a packed batch's arrays (the caller-built batch of
    include/lincheck.h: events, offsets, widths) and an lc_batch over them."""
    K = pk.n_keys
    n_ev = int(pk.ev_off[-1])
    arrs = dict(ev_off=pk.ev_off.copy(),
                events=pk.all_events(),
                trans=np.ctypeslib.as_array(pk.view.trans, shape=(int(pk.view.n_trans),)).copy(),
                width=np.ctypeslib.as_array(pk.view.key_width, shape=(K,)).copy(),
                states=np.ctypeslib.as_array(pk.view.key_states, shape=(K,)).copy())
    b = N.LcBatch()
    b.n_keys = K
    b.ev_off = N.ptr(arrs["ev_off"], C.c_uint64)
    b.events = N.ptr(arrs["events"], C.c_uint32)
    b.trans = N.ptr(arrs["trans"], C.c_uint32)
    b.n_trans = int(pk.view.n_trans)
    b.key_width = N.ptr(arrs["width"], C.c_uint8)
    b.key_states = N.ptr(arrs["states"], C.c_uint16)
    return arrs, b


def _check_batch(dev, b, K):
    arrs, r = dev._alloc(K)
    st = N.LcStats()
    N.check(N.lib().lc_check_batch(dev.handle, C.byref(b), C.byref(r), C.byref(st)))
    return arrs


def _expect_invalid(dev, b, K, key):
    with pytest.raises(N.LincheckError) as ei:
        _check_batch(dev, b, K)
    assert ei.value.code == -1 and f"key {key}" in str(ei.value), str(ei.value)
    h = C.c_void_p()
    N.check(N.lib().lc_upload(dev.handle, C.byref(b), C.byref(h)))  # T0-validated: uploads as it is
    try:
        valid, fe, cause = (np.zeros(K, np.int8), np.zeros(K, np.int32), np.zeros(K, np.uint8))
        r = N.LcResult(N.ptr(valid, C.c_int8), N.ptr(fe, C.c_int32), N.ptr(cause, C.c_uint8), None, None, None)
        st = N.LcStats()
        with pytest.raises(N.LincheckError) as ei:
            N.check(N.lib().lc_check_device(dev.handle, h, C.byref(r), 0, C.byref(st)))
        assert f"key {key}" in str(ei.value)  # (the result arrays of a refused call are unspecified)
    finally:
        N.lib().lc_dev_batch_free(h)


def test_t0_validates_events():
    """Every per-event malformation T0 checks, one at a time, on a batch of
    register-tier keys; after each refusal the same context checks the good
    batch bit-exactly."""
    h = H.synth(n_keys=300, ops_per_key=200, concurrency=6, anomaly_rate=0.1, seed=75)
    pk = Packed(h)
    K = pk.n_keys
    dev = Device(0)
    arrs, b = _batch_copy(pk)
    ev = arrs["events"]
    good = _check_batch(dev, b, K)
    _, orc = cref.check_history(h.as_c(), budget=dev.budget, threads=8)
    np.testing.assert_array_equal(good["valid"][:K], orc["valid"])

    def at(key, pred):
        lo, hi = int(pk.ev_off[key]), int(pk.ev_off[key + 1])
        return lo + int(np.flatnonzero(pred(ev[lo:hi]))[0])

    cases = []
    # an :ok of a slot with no pending op (the key's first event made an :ok)
    cases.append((211, at(211, lambda e: np.ones(len(e), bool)), lambda w: w | N.LC_EV_OK_BIT))
    # an :invoke into an occupied slot (the key's first :ok made an invoke)
    cases.append((57, at(57, lambda e: (e & N.LC_EV_OK_BIT) != 0), lambda w: (w & 0x7F000000)))
    # a transition id beyond the table
    cases.append((123, at(123, lambda e: (e & N.LC_EV_OK_BIT) == 0), lambda w: (w & 0xFF000000) | 0xFFFFF))
    # an :invoke in a slot >= 64 (a key declared to fit T0 cannot hold it)
    cases.append((290, at(290, lambda e: (e & N.LC_EV_OK_BIT) == 0), lambda w: (w & 0x80FFFFFF) | (70 << 24)))
    for key, j, mutate in cases:
        saved = int(ev[j])
        ev[j] = mutate(saved)
        _expect_invalid(dev, b, K, key)
        ev[j] = saved
        again = _check_batch(dev, b, K)
        np.testing.assert_array_equal(again["valid"][:K], good["valid"][:K])
        np.testing.assert_array_equal(again["fail_event"][:K], good["fail_event"][:K])


def test_spec_validates_large_batch():
    """The speculative segments' own validation (T0_STRICT blocks in the
    search launch) on a batch of more keys than one resident round of
    workgroups, where those blocks go first in the grid: every per-event
    malformation is refused naming its key, and between refusals the same
    context gives the oracle's records for the good batch."""
    h = H.synth(n_keys=3000, ops_per_key=300, concurrency=6, anomaly_rate=0.05, seed=81)
    pk = Packed(h)
    K = pk.n_keys
    dev = Device(0)
    arrs, b = _batch_copy(pk)
    ev = arrs["events"]
    _, orc = cref.check_history(h.as_c(), budget=dev.budget, threads=8)

    def node():
        out = np.zeros(K, np.uint64)
        st = N.LcStats()
        N.check(N.lib().lc_check_node(dev.handle, C.byref(b), K, N.ptr(out, C.c_uint64), C.byref(st)))
        return out, st

    rec, st = node()
    assert N.T0_PATH_NAMES.get(int(st.t0_path)) == "k_spec"
    v, c, fe = _decode(rec, K)
    np.testing.assert_array_equal(v, orc["valid"])
    np.testing.assert_array_equal(fe, orc["fail_event"])

    def at(key, pred):
        lo, hi = int(pk.ev_off[key]), int(pk.ev_off[key + 1])
        return lo + int(np.flatnonzero(pred(ev[lo:hi]))[0])

    cases = [
        (211, at(211, lambda e: np.ones(len(e), bool)), lambda w: w | N.LC_EV_OK_BIT),
        (1057, at(1057, lambda e: (e & N.LC_EV_OK_BIT) != 0), lambda w: (w & 0x7F000000)),
        (2123, at(2123, lambda e: (e & N.LC_EV_OK_BIT) == 0), lambda w: (w & 0xFF000000) | 0xFFFFF),
        (2890, at(2890, lambda e: (e & N.LC_EV_OK_BIT) == 0), lambda w: (w & 0x80FFFFFF) | (70 << 24)),
    ]
    for key, j, mutate in cases:
        saved = int(ev[j])
        ev[j] = mutate(saved)
        with pytest.raises(N.LincheckError) as ei:
            node()
        assert ei.value.code == -1 and f"key {key}" in str(ei.value), str(ei.value)
        ev[j] = saved
        again, _ = node()
        np.testing.assert_array_equal(again, rec)


def _ev16(w: int) -> int:
    """include/lincheck.h LC_EV16_*: a 32-bit event word in 16 bits (slot <= 15,
    transition id <= 2047)."""
    return ((w >> 16) & 0x8000) | (((w >> 24) & 0x7F) << 11) | (w & 0x7FF)


def test_spec_self_validates_staged_keys():
    """k_spec validates a key whose 16-bit words its block stages whole in LDS
    inside that block (its W waves, the slot protocol's state carried across
    their parts), not by a second HBM read in the validation blocks.  Each
    malformation the 16-bit words can carry, in keys early, in the middle and
    at the end of the batch and at a wave's part boundary, is refused naming
    its key; between refusals the same context gives the oracle's records."""
    h = H.synth(n_keys=1000, ops_per_key=300, concurrency=6, anomaly_rate=0.05, seed=83)
    pk = Packed(h)
    K = pk.n_keys
    assert pk.view.events16
    dev = Device(0)
    arrs, b = _batch_copy(pk)
    n_ev = int(pk.ev_off[-1])
    arrs["events16"] = np.ctypeslib.as_array(pk.view.events16, shape=(n_ev,)).copy()
    b.events16 = N.ptr(arrs["events16"], C.c_uint16)
    ev, e16 = arrs["events"], arrs["events16"]
    _, orc = cref.check_history(h.as_c(), budget=dev.budget, threads=8)

    def node():
        out = np.zeros(K, np.uint64)
        st = N.LcStats()
        N.check(N.lib().lc_check_node(dev.handle, C.byref(b), K, N.ptr(out, C.c_uint64), C.byref(st)))
        return out, st

    rec, st = node()
    assert N.T0_PATH_NAMES.get(int(st.t0_path)) == "k_spec"
    v, _, fe = _decode(rec, K)
    np.testing.assert_array_equal(v, orc["valid"])
    np.testing.assert_array_equal(fe, orc["fail_event"])

    def at(key, pred, frac=0.0):
        lo, hi = int(pk.ev_off[key]), int(pk.ev_off[key + 1])
        start = lo + int((hi - lo) * frac)
        return start + int(np.flatnonzero(pred(ev[start:hi]))[0])

    is_ok = lambda e: (e & N.LC_EV_OK_BIT) != 0  # noqa: E731
    is_inv = lambda e: (e & N.LC_EV_OK_BIT) == 0  # noqa: E731
    cases = [
        (3, at(3, lambda e: np.ones(len(e), bool)), lambda w: w | N.LC_EV_OK_BIT),   # :ok of a free slot
        (500, at(500, is_ok, 0.5), lambda w: w & 0x7F000000),                        # :invoke into a busy slot
        (501, at(501, is_ok, 0.26), lambda w: w & 0x7F000000),                       # near a wave's part boundary
        (998, at(998, is_inv, 0.9), lambda w: (w & 0xFF000000) | 0x7FF),              # transition id past the table
    ]
    for key, j, mutate in cases:
        saved, saved16 = int(ev[j]), int(e16[j])
        ev[j] = mutate(saved)
        e16[j] = _ev16(int(ev[j]))
        with pytest.raises(N.LincheckError) as ei:
            node()
        assert ei.value.code == -1 and f"key {key}" in str(ei.value), str(ei.value)
        ev[j], e16[j] = saved, saved16
        again, _ = node()
        np.testing.assert_array_equal(again, rec)


def test_t0_refuses_understated_width():
    """key_width claims fewer ops pending at once than a key has: the batch is
    declared register-tier-only, T0 meets the 11th pending op, and the key is
    refused instead of being spilled to a tier that is never launched."""
    h = H.synth(n_keys=40, ops_per_key=400, concurrency=14, seed=76)
    pk = Packed(h)
    K = pk.n_keys
    dev = Device(0)
    arrs, b = _batch_copy(pk)
    wide = np.flatnonzero(arrs["width"] > 10)
    assert wide.size > 0
    arrs["width"][:] = np.minimum(arrs["width"], 10)
    with pytest.raises(N.LincheckError) as ei:
        _check_batch(dev, b, K)
    assert ei.value.code == -1 and "understate" in str(ei.value)
    device_vs_oracle(h, dev)


def test_async_errors_surface_at_wait():
    """An asynchronous resident step over a malformed T0-validated batch:
    the refusal comes from lc_wait."""
    h = H.synth(n_keys=300, ops_per_key=200, concurrency=6, seed=77)
    pk = Packed(h)
    K = pk.n_keys
    dev = Device(0)
    arrs, b = _batch_copy(pk)
    j = int(pk.ev_off[99])
    arrs["events"][j] |= N.LC_EV_OK_BIT
    h_db = C.c_void_p()
    N.check(N.lib().lc_upload(dev.handle, C.byref(b), C.byref(h_db)))
    try:
        st = N.LcStats()
        N.check(N.lib().lc_check_node_device(dev.handle, h_db, K, N.LC_DEV_ASYNC, C.byref(st)))
        with pytest.raises(N.LincheckError) as ei:
            dev.wait()
        assert "key 99" in str(ei.value)
    finally:
        N.lib().lc_dev_batch_free(h_db)
    device_vs_oracle(h, dev)


def test_pipelined_step_error_surfaces_at_wait_step():
    """A malformed batch in a pipelined node step (lc_check_node_async): the
    refusal comes from the lc_wait_step that waits for that step, naming the
    key; the error is then cleared, and the next steps are bit-exact."""
    from lincheck.checker import PinnedRecords
    h = H.synth(n_keys=300, ops_per_key=200, concurrency=6, anomaly_rate=0.1, seed=79)
    pk = Packed(h)
    K = pk.n_keys
    dev = Device(0)
    arrs, b = _batch_copy(pk)
    arrs["events"][int(pk.ev_off[137])] |= N.LC_EV_OK_BIT
    bad = PinnedRecords(K)
    st = N.LcStats()
    rc = N.check(N.lib().lc_check_node_async(dev.handle, C.byref(b), K, N.ptr(bad, C.c_uint64), C.byref(st)))
    assert rc == 1  # enqueued
    with pytest.raises(N.LincheckError) as ei:
        dev.wait_step(0)
    assert ei.value.code == -1 and "key 137" in str(ei.value), str(ei.value)
    assert dev.wait()[0] >= 0  # nothing left to report
    _, orc = cref.check_history(h.as_c(), budget=dev.budget, threads=8)
    for _ in range(2):
        good = PinnedRecords(K)
        assert dev.check_node_async(pk, K, good)[0]
        dev.wait_step(0)
        v, _, fe = _decode(np.asarray(good), K)
        np.testing.assert_array_equal(v, orc["valid"])
        np.testing.assert_array_equal(fe, orc["fail_event"])


def test_two_malformed_pipelined_steps_report_their_own_keys():
    """Two malformed batches enqueued back to back: each step
    has its own error words, read and cleared atomically by the wait for
    that step, so the first wait names the first step's key, the second
    wait the second's -- neither refusal is lost or blamed on the other
    step -- and nothing is left for lc_wait."""
    from lincheck.checker import PinnedRecords
    h = H.synth(n_keys=300, ops_per_key=200, concurrency=6, seed=81)
    pk = Packed(h)
    K = pk.n_keys
    dev = Device(0)
    steps = []
    for bad_key in (40, 211):
        arrs, b = _batch_copy(pk)
        arrs["events"][int(pk.ev_off[bad_key])] |= N.LC_EV_OK_BIT
        out = PinnedRecords(K)
        st = N.LcStats()
        rc = N.check(N.lib().lc_check_node_async(dev.handle, C.byref(b), K, N.ptr(out, C.c_uint64), C.byref(st)))
        assert rc == 1  # enqueued
        steps.append((arrs, b, out))
    for back, bad_key in ((1, 40), (0, 211)):
        with pytest.raises(N.LincheckError) as ei:
            dev.wait_step(back)
        assert ei.value.code == -1 and f"key {bad_key}" in str(ei.value), str(ei.value)
    assert dev.wait()[0] >= 0  # nothing left to report
    _, orc = cref.check_history(h.as_c(), budget=dev.budget, threads=8)
    good = PinnedRecords(K)
    assert dev.check_node_async(pk, K, good)[0]
    dev.wait_step(0)
    v, _, fe = _decode(np.asarray(good), K)
    np.testing.assert_array_equal(v, orc["valid"])
    np.testing.assert_array_equal(fe, orc["fail_event"])


def test_many_keys_take_the_unsegmented_tier():
    """A batch of 400,000 small keys: the speculative segments would need
    ~9.6 GB of per-key workspace, so the step takes the
    unsegmented register tier (workspace per resident wave) -- verdicts and
    failing events still the oracle's."""
    h = H.synth(n_keys=400_000, ops_per_key=3, concurrency=2, anomaly_rate=0.01, seed=83)
    pk = Packed(h)
    res = Device(0).check(pk, verdicts_only=True)
    assert res.stats["t0_path"] == "k_search_lattice"
    _, orc = cref.check_history(h.as_c(), budget=1 << 20, threads=8)
    np.testing.assert_array_equal(res.valid, orc["valid"])
    np.testing.assert_array_equal(res.fail_event, orc["fail_event"])


def test_two_rank_node_step(tmp_path):
    """E-1 (independent/checker's pmap, etcdemo.clj:115) with two ranks: two
    fresh processes on the one GPU, each running the library's node step
    (lc_check_node) on its shard of a mixed batch -- 4,001 C5-shaped keys and
    6 C4-shaped ones -- split by estimated cost (parallel.key_costs /
    cost_shards: the C4-shaped keys by LPT, the rest in contiguous runs),
    their blocks of LC_REC_* records all-gathered over gloo in rank order.
    The node's records, put back in the caller's key order
    (parallel.node_key_order; the padding of the shorter shard must be 0),
    equal the oracle's for every key and a single-process check of the same
    batch (devices=[0, 0]); the ranks' estimated costs are within 10 %."""
    import socket
    import subprocess
    import sys
    from lincheck import parallel as P
    from node_rank_main import BUDGET, mixed_history
    n_keys, ops, world = 4001, 300, 2
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    out = str(tmp_path / "node.npy")
    helper = os.path.join(os.path.dirname(os.path.abspath(__file__)), "node_rank_main.py")
    procs = [subprocess.Popen([sys.executable, helper, str(r), str(world), str(port), str(n_keys), str(ops), out])
             for r in range(world)]
    try:
        for p in procs:
            assert p.wait(timeout=240) == 0
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    node = np.load(out)
    h = mixed_history(n_keys, ops)
    keys, costs = P.key_costs(h, BUDGET)
    shards = P.cost_shards(costs, world)
    block = max(len(s) for s in shards)
    loads = P.shard_costs(costs, shards)
    assert loads.max() <= 1.1 * loads.min()
    assert node.size == block * world
    v, c, fe = P.node_key_order(node, shards, block)
    _, orc = cref.check_history(h.as_c(), budget=BUDGET, threads=8)
    np.testing.assert_array_equal(v, orc["valid"])
    np.testing.assert_array_equal(c, orc["cause"])
    np.testing.assert_array_equal(fe, orc["fail_event"])
    assert (v == 0).sum() > 10
    one = Device(0, devices=[0, 0], budget=BUDGET).check(Packed(h), verdicts_only=True)
    np.testing.assert_array_equal(one.valid, v)
    np.testing.assert_array_equal(one.fail_event, fe)


def test_chunked_node_step_names_the_batch_key():
    """A malformed key in the third of four upload chunks of lc_check_node:
    the error names its index in the caller's batch, not in its chunk."""
    h = H.synth(n_keys=400, ops_per_key=200, concurrency=6, seed=80)
    pk = Packed(h)
    K = pk.n_keys
    dev = Device(0, path_flags=N.LC_PATH_CHUNKS_ON)
    arrs, b = _batch_copy(pk)
    arrs["events"][int(pk.ev_off[263])] |= N.LC_EV_OK_BIT
    out = np.zeros(K, np.uint64)
    with pytest.raises(N.LincheckError) as ei:
        N.check(N.lib().lc_check_node(dev.handle, C.byref(b), K, N.ptr(out, C.c_uint64), None))
    assert "key 263" in str(ei.value), str(ei.value)
    rec, _ = dev.check_node(pk, K)
    _, orc = cref.check_history(h.as_c(), budget=dev.budget, threads=8)
    np.testing.assert_array_equal(_decode(rec, K)[0], orc["valid"])


def test_wait_step_waits_for_the_step_asked():
    """lc_wait_step(1) returns once the step before the latest is done: step
    A's records (one node buffer per step would be overwritten, so A and B
    write different result arrays) are final while B may still run."""
    from test_gpu_parity import _HipBuf
    dev = Device(0)
    hA = H.synth(n_keys=500, ops_per_key=600, concurrency=10, anomaly_rate=0.1, seed=78)
    hB = H.synth(n_keys=500, ops_per_key=600, concurrency=10, anomaly_rate=0.1, seed=79)
    outs = []
    for h in (hA, hB):
        pk = Packed(h)
        K = pk.n_keys
        bufs = (_HipBuf(K), _HipBuf(4 * K), _HipBuf(K))
        for x in bufs:
            x.fill(0x5A)
        r = N.LcResult(C.cast(bufs[0].ptr, N.P(C.c_int8)), C.cast(bufs[1].ptr, N.P(C.c_int32)),
                       C.cast(bufs[2].ptr, N.P(C.c_uint8)), None, None, None)
        outs.append((h, dev.upload(pk), bufs, r))
    dev.wait()
    for _, db, _, r in outs:
        db.check_into(r, asynchronous=True)
    dev.wait_step(1)
    _, orcA = cref.check_history(hA.as_c(), budget=dev.budget, threads=8)
    np.testing.assert_array_equal(outs[0][2][0].get(np.int8), orcA["valid"])
    np.testing.assert_array_equal(outs[0][2][1].get(np.int32), orcA["fail_event"])
    n, _ = dev.wait()
    assert n == 2
    _, orcB = cref.check_history(hB.as_c(), budget=dev.budget, threads=8)
    np.testing.assert_array_equal(outs[1][2][0].get(np.int8), orcB["valid"])


@pytest.mark.parametrize("forced", [True, False])
def test_node_chunked_upload_pipeline(forced):
    """lc_check_node on a large register-tier shard: key chunks uploaded on a
    stream of their own, each chunk's search waiting for its own copy.  The
    records equal the one-launch check (LC_PATH_CHUNKS_OFF), and the oracle's
    verdicts.  forced: a small C5-shaped shard chunked by LC_PATH_CHUNKS_ON;
    otherwise a C3-shard-sized one (4,096+ keys, 8M+ events) chunked by
    default."""
    if forced:
        h = H.synth(n_keys=500, ops_per_key=300, concurrency=10, anomaly_rate=0.1, seed=73)
    else:
        h = H.synth(n_keys=6000, ops_per_key=800, concurrency=10, anomaly_rate=0.02, seed=74)
    pk = Packed(h)
    K = pk.n_keys
    dev = Device(0, path_flags=N.LC_PATH_CHUNKS_ON if forced else 0)
    rec, _ = dev.check_node(pk, K)
    for _ in range(2):  # repeated steps reuse the chunk batches
        rec2, _ = dev.check_node(pk, K)
        np.testing.assert_array_equal(rec2, rec)
    one, _ = Device(0, path_flags=N.LC_PATH_CHUNKS_OFF).check_node(pk, K)
    np.testing.assert_array_equal(rec, one)
    v, c, fe = _decode(rec, K)
    keys, orc = cref.check_history(h.as_c(), budget=1 << 20, threads=8)
    np.testing.assert_array_equal(v, orc["valid"])
    np.testing.assert_array_equal(fe, orc["fail_event"])
    assert (v == 0).any()


def test_device_validates_batches_beyond_the_register_tier():
    """A batch whose keys leave the register tier (crashed ops: 12-20 ops
    pending, the LDS and HBM set tiers run) is validated on the device too
    (k_validate<true> beside T0; the set tiers do nothing over a refused
    batch): each malformation is refused naming its key, on the host-to-host
    and the resident path, and the context then checks the good batch
    bit-exactly."""
    h = H.synth(n_keys=48, ops_per_key=400, concurrency=14, info_rate=0.01, anomaly_rate=0.2, seed=78)
    pk = Packed(h)
    K = pk.n_keys
    dev = Device(0)
    arrs, b = _batch_copy(pk)
    assert (arrs["width"] > 10).any()  # not a register-tier batch
    ev = arrs["events"]
    good = _check_batch(dev, b, K)
    _, orc = cref.check_history(h.as_c(), budget=dev.budget, threads=8)
    np.testing.assert_array_equal(good["valid"][:K], orc["valid"])
    np.testing.assert_array_equal(good["fail_event"][:K], orc["fail_event"])

    def at(key, pred):
        lo, hi = int(pk.ev_off[key]), int(pk.ev_off[key + 1])
        return lo + int(np.flatnonzero(pred(ev[lo:hi]))[0])

    wide_key = int(np.flatnonzero(arrs["width"] > 10)[0])
    cases = [
        (11, at(11, lambda e: np.ones(len(e), bool)), lambda w: w | N.LC_EV_OK_BIT),        # :ok of no pending op
        (23, at(23, lambda e: (e & N.LC_EV_OK_BIT) != 0), lambda w: (w & 0x7F000000)),       # :invoke into a held slot
        (37, at(37, lambda e: (e & N.LC_EV_OK_BIT) == 0), lambda w: (w & 0xFF000000) | 0xFFFFF),  # transition id
        (wide_key, at(wide_key, lambda e: (e & N.LC_EV_OK_BIT) == 0),                          # slot past key_width
         lambda w: (w & 0x80FFFFFF) | (100 << 24)),
    ]
    for key, j, mutate in cases:
        saved = int(ev[j])
        ev[j] = mutate(saved)
        _expect_invalid(dev, b, K, key)
        ev[j] = saved
        again = _check_batch(dev, b, K)
        np.testing.assert_array_equal(again["valid"][:K], good["valid"][:K])
        np.testing.assert_array_equal(again["fail_event"][:K], good["fail_event"][:K])


@pytest.mark.parametrize("rccl", [False, True])
def test_pipelined_node_steps_bit_exact(rccl):
    """lc_check_node_async: batches of different sizes in flight two at a
    time (each step's upload overlapping the previous search, the staging
    slots used in turn), every step's records in its own page-locked buffer;
    after the wait each equals lc_check_node's.  Without a communicator the
    search writes the records into that buffer itself; with a (one-rank) RCCL
    communicator they go through the all-gather and a download.  A batch
    beyond the register tier runs synchronously, and a pageable caller batch
    goes through the staging copy."""
    from lincheck.checker import PinnedRecords
    shapes = [dict(n_keys=300, ops_per_key=400, concurrency=10, anomaly_rate=0.1, seed=81),
              dict(n_keys=120, ops_per_key=900, concurrency=8, anomaly_rate=0.2, seed=82),
              dict(n_keys=1000, ops_per_key=200, concurrency=10, seed=83)]
    pks = [Packed(H.synth(**s)) for s in shapes]
    dev = Device(0, comm=(0, 1, comm_id()) if rccl else None)
    refs = [dev.check_node(pk, pk.n_keys + 3)[0].copy() for pk in pks]
    seq = [0, 1, 2, 0, 2, 1, 1, 0, 2, 2, 0, 1]
    bufs = [PinnedRecords(pks[i].n_keys + 3) for i in seq]
    enq = [dev.check_node_async(pks[i], pks[i].n_keys + 3, buf)[0] for i, buf in zip(seq, bufs)]
    assert all(enq)
    n, _ = dev.wait()
    assert n == len(seq)
    for i, buf in zip(seq, bufs):
        np.testing.assert_array_equal(np.asarray(buf), refs[i])
    # beyond the register tier: runs as lc_check_node
    pk = Packed(H.synth(**SHAPES["crashed"]))
    buf = PinnedRecords(pk.n_keys)
    e, _ = dev.check_node_async(pk, pk.n_keys, buf)
    assert not e
    np.testing.assert_array_equal(np.asarray(buf), dev.check_node(pk, pk.n_keys)[0])
    # a pageable caller batch (staged), then an error surfacing at the wait
    h = H.synth(n_keys=300, ops_per_key=200, concurrency=6, seed=84)
    pk = Packed(h)
    arrs, b = _batch_copy(pk)
    ref = dev.check_node(pk, pk.n_keys)[0].copy()
    outs = [PinnedRecords(pk.n_keys) for _ in range(3)]
    for o in outs:
        N.check(N.lib().lc_check_node_async(dev.handle, C.byref(b), pk.n_keys, N.ptr(o, C.c_uint64), None))
    dev.wait()
    for o in outs:
        np.testing.assert_array_equal(np.asarray(o), ref)
    arrs["events"][int(pk.ev_off[42])] |= N.LC_EV_OK_BIT
    N.check(N.lib().lc_check_node_async(dev.handle, C.byref(b), pk.n_keys, N.ptr(outs[0], C.c_uint64), None))
    with pytest.raises(N.LincheckError) as ei:
        dev.wait()
    assert "key 42" in str(ei.value)
    device_vs_oracle(h, dev)


def test_c3_full_key_space_eight_shards():
    """BASELINE C3's whole key space (100,000 keys x 2,000 ops, concurrency
    10; 0.1 % of keys corrupted) through a context of eight key shards on
    this one GPU (devices [0] * 8: the node's 8-GPU split, one stream and
    scratch per shard), the pmap at etcdemo.clj:115 as the 8-GPU node runs
    it.  Properties at full size: every uncorrupted key is valid (the
    generator's histories are linearizable by construction) and every
    invalid key is a corrupted one; the first shard's records -- the keys one
    GPU of the node checks -- equal the oracle's, and the node step on
    eight contiguous shards gives the same verdicts as the whole batch."""
    h = H.synth(n_keys=100_000, ops_per_key=2000, concurrency=10, anomaly_rate=0.001, seed=3)
    pk = Packed(h)
    K = pk.n_keys
    assert K == 100_000
    res = Device(0, devices=[0] * 8).check(pk, verdicts_only=True)
    bad = np.zeros(K, bool)
    idx = {k: i for i, k in enumerate(pk.keys)}
    for k in h.anomalous_keys:
        bad[idx[k]] = True
    assert bad.sum() > 50
    assert (res.valid[~bad] == 1).all() and (res.fail_event[~bad] == -1).all()
    assert (res.valid[res.valid != 1] == 0).all()  # no key :unknown
    assert bad[res.valid == 0].all() and (res.valid == 0).sum() > 0
    # the first of the eight shards against the oracle (12,500 keys)
    e = int(pk.ev_off[K // 8])
    assert e > 0
    sub = H.synth(n_keys=K // 8, ops_per_key=2000, concurrency=10, anomaly_rate=0.001, seed=3)
    _, orc = cref.check_history(sub.as_c(), budget=1 << 20, threads=16)
    np.testing.assert_array_equal(res.valid[:K // 8], orc["valid"])
    np.testing.assert_array_equal(res.fail_event[:K // 8], orc["fail_event"])
    # the node step over the same key space as eight rank-shards (the
    # records the 8-GPU all-gather assembles), one after another on this GPU
    dev = Device(0)
    for r in range(8):
        k0, k1 = P.shard_range(K, 8, r)
        shard = Packed(H.synth(n_keys=k1 - k0, ops_per_key=2000, concurrency=10, anomaly_rate=0.001, seed=3,
                               key_base=k0))
        rec, _ = dev.check_node(shard, -(-K // 8))
        v, _, fe = _decode(rec, k1 - k0)
        np.testing.assert_array_equal(v, res.valid[k0:k1])
        np.testing.assert_array_equal(fe, res.fail_event[k0:k1])
