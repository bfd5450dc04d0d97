"""Device search vs the C restatement of knossos.linear -- bit-exact parity.

Every case runs the same seeded history through liblincheck.so (the HIP
path) and oracle/linear_ref.c and compares, per key: :valid?, the cause, the
failing event, the peak config-set size, and the total probe count.
"""
import numpy as np
import pytest

import cref
from helpers import device_vs_oracle
from lincheck import history as H
from lincheck.checker import Device

pytestmark = pytest.mark.gpu


def test_c2_shape_all_valid(device):
    h = H.synth(n_keys=300, ops_per_key=1000, concurrency=10, seed=2)
    _, res, _ = device_vs_oracle(h, device)
    assert (res.valid == 1).all()


def test_c5_shape_anomalies(device):
    h = H.synth(n_keys=400, ops_per_key=1000, concurrency=10, anomaly_rate=0.05, seed=5)
    _, res, _ = device_vs_oracle(h, device)
    assert (res.valid == 0).sum() > 0


def test_small_keys_many(device):
    h = H.synth(n_keys=3000, ops_per_key=40, concurrency=5, anomaly_rate=0.2, seed=11)
    device_vs_oracle(h, device)


def test_tight_budget_unknown(device):
    dev = Device(0, budget=48)
    h = H.synth(n_keys=200, ops_per_key=500, concurrency=10, anomaly_rate=0.1, seed=13)
    _, res, _ = device_vs_oracle(h, dev, budget=48)
    assert (res.valid == -1).sum() > 0


def test_high_concurrency_spills_to_t2(device):
    h = H.synth(n_keys=64, ops_per_key=600, concurrency=16, seed=17)
    _, res, _ = device_vs_oracle(h, device)


def test_c4_shape_crashed_ops_wide(device):
    """Crashed (:info) write/cas ops stay callable forever: frontier blow-up,
    > 56 window slots (wide configs, HBM tier), budget -> :unknown."""
    dev = Device(0, budget=1 << 14)
    h = H.synth(n_keys=24, ops_per_key=2000, concurrency=30, info_rate=0.02, seed=4)
    _, res, _ = device_vs_oracle(h, dev, budget=1 << 14)
    assert (res.valid == -1).sum() > 0


@pytest.mark.parametrize("conc,info,budget", [(20, 0.005, 1 << 20), (16, 0.01, 1 << 20), (16, 0.01, 8192),
                                               (16, 0.01, 1000)])
def test_hbm_tier_narrow_lds_and_hbm_passes(device, conc, info, budget):
    """Crashed ops, sets of 10^3-10^5 configs: keys reach the HBM tier with
    narrow configs, where small :oks keep their hash sets in LDS and larger
    ones are redone on the HBM tables.  Keys finish (valid / invalid) at the
    full budget, so peaks and probe counts are compared too; the smaller
    budgets stop inside an LDS pass (1000) and after a redo (8192)."""
    dev = Device(0, budget=budget, count_probes=True)
    h = H.synth(n_keys=32, ops_per_key=600, concurrency=conc, info_rate=info, anomaly_rate=0.1, seed=31)
    _, res, orc = device_vs_oracle(h, dev, budget=budget)
    if budget >= 8192:
        assert res.stats["deep_keys"] > 0  # keys the HBM tier searched
    else:  # the budget ends keys before they outgrow the LDS tiers
        assert (orc["cause"] == 2).any()
    if budget == 1 << 20:
        assert (orc["cause"] != 2).all() and orc["peak"].max() > 2048


def test_many_register_values_wide(device):
    """> 255 distinct register values in a key: per-key state tables, wide configs."""
    h = H.synth(n_keys=32, ops_per_key=600, concurrency=8, n_values=5000, anomaly_rate=0.2, seed=21)
    device_vs_oracle(h, device)


def test_window_overflow(device):
    """More than 112 ops pending at once -> :unknown (cause window), as the oracle."""
    from lincheck.independent import Tuple
    ops = []
    for p in range(120):
        ops.append({"type": "invoke", "f": "read", "value": Tuple(0, None), "process": p})
    ops.append({"type": "ok", "f": "read", "value": Tuple(0, None), "process": 0})
    ops.append({"type": "invoke", "f": "write", "value": Tuple(1, 3), "process": 500})
    ops.append({"type": "ok", "f": "write", "value": Tuple(1, 3), "process": 500})
    _, res, _ = device_vs_oracle(H.History.from_ops(ops), device)
    assert list(res.valid) == [-1, 1]
    assert list(res.cause) == [3, 0]


@pytest.mark.parametrize("mname", ["mutex", "register"])
def test_other_models(device, mname):
    """(model/mutex) and (model/register) on the same kernels (SURVEY.md 8(f)
    F-4): bit-exact verdicts, failing events and peak set sizes."""
    import cref
    from histgen import mutex_history, random_history
    from lincheck import model
    from lincheck.checker import Packed
    mdl = {"mutex": model.mutex(), "register": model.register()}[mname]
    if mname == "mutex":
        ops = mutex_history(3, n_keys=400, rounds=60, procs=8)
    else:
        ops = random_history(77, n_keys=200, max_ops=60, procs=10, model=mname, p_garbage_read=0.05,
                             p_open=0.0, p_info=0.05)
    h = H.History.from_ops(ops)
    pk = Packed(h, mdl)
    res = device.check(pk)
    keys, orc = cref.check_history(h.as_c(), model=mname, threads=8)
    assert list(keys) == pk.keys
    np.testing.assert_array_equal(res.valid, orc["valid"])
    np.testing.assert_array_equal(res.fail_event, orc["fail_event"])
    np.testing.assert_array_equal(res.peak, orc["peak"])
    assert (res.valid == 1).any() and (res.valid == 0).any()


@pytest.mark.parametrize("peaks", [True, False])
@pytest.mark.parametrize("shape", ["lattice", "wide_window", "mutex"])
def test_counterexamples(device, shape, peaks):
    """:configs and :final-paths of invalid keys from the
    device's final config records, against the restatement's final config set
    and its full path enumeration: the device's (first <= 10) configs and the
    paths built from them are subsets, and equal when the restatement has no
    more than 10 of each."""
    import linear_ref as LR
    from helpers import config_tuple, path_tuple
    from histgen import mutex_history
    from lincheck import model
    from lincheck.checker import Packed, _render_key
    mname = "mutex" if shape == "mutex" else "cas-register"
    if shape == "lattice":      # <= 10 pending: the register-lattice tier
        h = H.synth(n_keys=300, ops_per_key=80, concurrency=6, anomaly_rate=0.3, seed=31)
    elif shape == "wide_window":  # 12-16 pending: the LDS / HBM set tiers
        h = H.synth(n_keys=150, ops_per_key=120, concurrency=14, anomaly_rate=0.3, seed=32)
    else:
        h = H.History.from_ops(mutex_history(5, n_keys=200, rounds=30, procs=6, corrupt=0.3))
    mdl = model.mutex() if mname == "mutex" else model.cas_register()
    ops = h.to_ops()
    pk = Packed(h, mdl)
    # peaks=False: final configs only, as the Jepsen-shaped checkers ask
    # (the register tier's exact speculative segments)
    res = device.check(pk, peaks=peaks)
    n_bad = 0
    for i, k in enumerate(pk.keys):
        if res.valid[i] != 0:
            continue
        sub = LR.subhistory(ops, k)
        a = LR.analysis(sub, model=mname)
        assert a.valid is False and a.fail_event == res.fail_event[i]
        m = _render_key(pk, i, res, None)
        exp_cfgs = {(bool(st) if mname == "mutex" else st,
                     frozenset(sub[a.ops[q].invoke_pos]["index"] for q in L)) for st, L in a.final_configs}
        got_cfgs = [config_tuple(c, mname) for c in m["configs"]]
        assert len(set(got_cfgs)) == len(got_cfgs) == min(10, len(exp_cfgs)), f"key {k}"
        assert set(got_cfgs) <= exp_cfgs, f"key {k}"
        exp_paths = LR.final_paths(a, sub, mname)
        got_paths = {path_tuple(p, mname) for p in m["final-paths"]}
        assert len(got_paths) == len(m["final-paths"]) > 0
        if exp_paths is None:   # too many to enumerate: 10 distinct paths
            assert len(got_paths) == 10
            continue
        assert got_paths <= exp_paths, f"key {k}"
        if len(exp_cfgs) <= 10 and len(exp_paths) <= 10:
            assert got_paths == exp_paths, f"key {k}"
        n_bad += 1
    assert n_bad > 5


def test_compact_t0_build_heavy_widths(device):
    """More keys than SIMD slots: T0's compact build (4 lattice registers, 9-10
    pending ops in the LDS workspace) on keys up to 10 ops wide.  Smaller
    batches take the wide build (16 registers); both must match the oracle."""
    h = H.synth(n_keys=2600, ops_per_key=120, concurrency=10, anomaly_rate=0.1, seed=41)
    _, res, _ = device_vs_oracle(h, device)
    assert (res.valid == 0).any()


@pytest.mark.parametrize("shape", ["c2", "c5", "compact_heavy", "high_concurrency", "many_values"])
def test_verdicts_only_fast_path(shape):
    """Verdict-only requests take T0's fast path (the compact build keeps its
    lane lattice closed under the pending ops instead of holding Knossos's
    exact set); verdicts, causes and failing events must stay bit-exact."""
    dev = Device(0)  # no probe counting: the fast path is eligible
    h = {
        "c2": lambda: H.synth(n_keys=300, ops_per_key=1000, concurrency=10, seed=2),
        "c5": lambda: H.synth(n_keys=400, ops_per_key=1000, concurrency=10, anomaly_rate=0.05, seed=5),
        "compact_heavy": lambda: H.synth(n_keys=2600, ops_per_key=120, concurrency=10, anomaly_rate=0.1, seed=41),
        "high_concurrency": lambda: H.synth(n_keys=64, ops_per_key=600, concurrency=16, seed=17),
        "many_values": lambda: H.synth(n_keys=32, ops_per_key=600, concurrency=8, n_values=5000,
                                       anomaly_rate=0.2, seed=21),
    }[shape]()
    device_vs_oracle(h, dev, verdicts_only=True)


class _HipBuf:
    """Device memory from the HIP runtime liblincheck itself links (a second
    runtime -- torch's -- must not initialise the GPU after this one)."""
    _rt = None

    def __init__(self, nbytes: int):
        import ctypes as C
        if _HipBuf._rt is None:
            _HipBuf._rt = C.CDLL("libamdhip64.so.7")
        self.C, self.n = C, nbytes
        self.ptr = C.c_void_p()
        assert self._rt.hipMalloc(C.byref(self.ptr), C.c_size_t(nbytes)) == 0

    def fill(self, byte: int):
        assert self._rt.hipMemset(self.ptr, self.C.c_int(byte), self.C.c_size_t(self.n)) == 0

    def get(self, dtype) -> np.ndarray:
        out = np.empty(self.n // np.dtype(dtype).itemsize, dtype)
        assert self._rt.hipMemcpy(out.ctypes.data_as(self.C.c_void_p), self.ptr, self.C.c_size_t(self.n), 2) == 0
        return out

    def __del__(self):
        if self._rt is not None and self.ptr:
            self._rt.hipFree(self.ptr)


@pytest.mark.parametrize("shape", ["c5", "high_concurrency", "many_values", "crashed"])
def test_resident_device_results(device, shape):
    """The bench's path: a batch resident in HBM, verdicts written to caller
    device arrays (lc_check_device with dev_result).  When no key can leave
    T0 the step is T0 alone (no T1/T2 launches, no counter readback); the
    other shapes take the full tier chain.  Repeated steps on one batch must
    keep giving the oracle's verdicts and failing events."""
    import ctypes as C

    import cref
    from lincheck import _native as N
    from lincheck.checker import Packed

    h = {
        "c5": lambda: H.synth(n_keys=400, ops_per_key=1000, concurrency=10, anomaly_rate=0.05, seed=5),
        "high_concurrency": lambda: H.synth(n_keys=64, ops_per_key=600, concurrency=16, seed=17),
        "many_values": lambda: H.synth(n_keys=32, ops_per_key=600, concurrency=8, n_values=5000,
                                       anomaly_rate=0.2, seed=21),
        "crashed": lambda: H.synth(n_keys=32, ops_per_key=600, concurrency=16, info_rate=0.01, anomaly_rate=0.1,
                                   seed=31),
    }[shape]()
    packed = Packed(h)
    dev = Device(0)
    db = dev.upload(packed)
    K = packed.n_keys
    valid, fev, cause = _HipBuf(K), _HipBuf(4 * K), _HipBuf(K)
    r = N.LcResult(C.cast(valid.ptr, N.P(C.c_int8)), C.cast(fev.ptr, N.P(C.c_int32)),
                   C.cast(cause.ptr, N.P(C.c_uint8)), None, None, None)
    _, orc = cref.check_history(h.as_c(), budget=dev.budget, threads=8)
    for _ in range(3):
        for b in (valid, fev, cause):
            b.fill(0x5A)
        st = db.check_into(r)
        np.testing.assert_array_equal(valid.get(np.int8), orc["valid"])
        np.testing.assert_array_equal(fev.get(np.int32), orc["fail_event"])
        np.testing.assert_array_equal(cause.get(np.uint8), orc["cause"])
    if shape == "c5":
        assert st.deep_keys == 0


def test_c3_shard_scale(device):
    """One GPU's C3 shard at 8 GPUs (12,500 keys x 2,000 ops = 25 M ops, the
    compact T0 build with many keys per SIMD), with 0.5 % of keys corrupted:
    bit-exact against the oracle on every key, plus the generator's
    size-independent property -- a key that was not corrupted is
    linearizable by construction, so every invalid key is a corrupted one."""
    h = H.synth(n_keys=12_500, ops_per_key=2000, concurrency=10, anomaly_rate=0.005, seed=3)
    packed, res, orc = device_vs_oracle(h, Device(0), verdicts_only=True)
    bad = set(h.anomalous_keys)
    keys = np.array(packed.keys)
    assert set(keys[res.valid == 0]) <= bad
    assert (res.valid[~np.isin(keys, list(bad))] == 1).all()
    assert (res.valid == 0).sum() > 0


def test_degenerate_histories(device):
    """Edge cases of the demo's check, end to end through
    independent/checker(linearizable): an empty history, nemesis ops only,
    an op that never returns, a failed op only (its pair is dropped, so the
    key has no events), and a crashed write that must be linearized for a
    later read.  Each result map must agree with the oracle's verdicts."""
    from lincheck import checker as ck
    from lincheck import independent, model
    from lincheck.independent import Tuple

    def op(t, f, v, p):
        return {"type": t, "f": f, "value": v, "process": p}

    nem = op("info", "start", None, "nemesis")
    cases = {
        "empty": ([], True, []),
        "nemesis_only": ([nem, op("info", "stop", None, "nemesis")], True, []),
        "never_returns": ([op("invoke", "read", Tuple(0, None), 0)], True, []),
        "failed_only": ([op("invoke", "write", Tuple(0, 1), 0), op("fail", "write", Tuple(0, 1), 0)], True, []),
        "crashed_write_read_later": ([op("invoke", "write", Tuple(0, 3), 0), op("info", "write", Tuple(0, 3), 0),
                                      op("invoke", "read", Tuple(0, None), 1), op("ok", "read", Tuple(0, 3), 1)],
                                     True, []),
        "stale_read_two_keys": ([op("invoke", "write", Tuple(0, 3), 0), op("ok", "write", Tuple(0, 3), 0),
                                 op("invoke", "read", Tuple(0, None), 1), op("ok", "read", Tuple(0, 4), 1),
                                 op("invoke", "write", Tuple(1, 2), 2), op("ok", "write", Tuple(1, 2), 2), nem],
                                False, [0]),
    }
    chk = independent.checker(ck.linearizable({"model": model.cas_register(), "algorithm": "linear"}))
    for name, (ops, valid, failures) in cases.items():
        out = chk.check({}, ops, {})
        assert out["valid?"] is valid, name
        assert sorted(out["failures"]) == failures, name
        if ops:
            h = H.History.from_ops(ops)
            keys, orc = cref.check_history(h.as_c(), budget=1 << 20)
            assert sorted(k for k, r in zip(keys, orc) if r["valid"] == 0) == failures, name


def test_check_batch_staging_reuse():
    """lc_check_batch keeps its device arrays across calls (grown on demand):
    batches that shrink, grow and switch models on ONE context stay bit-exact
    with the oracle, and a batch re-checked after others gives the same answer."""
    from histgen import mutex_history
    from lincheck import model
    from lincheck.checker import Packed
    dev = Device(0)
    seq = [H.synth(n_keys=200, ops_per_key=800, concurrency=10, anomaly_rate=0.05, seed=31),
           H.synth(n_keys=7, ops_per_key=30, concurrency=4, anomaly_rate=0.3, seed=32),
           None,  # mutex batch (per-model transition table) in between
           H.synth(n_keys=500, ops_per_key=1200, concurrency=12, anomaly_rate=0.05, seed=33)]
    first = None
    for h in seq:
        if h is None:
            hm = H.History.from_ops(mutex_history(5, n_keys=50, rounds=30, procs=6))
            pk = Packed(hm, model.mutex())
            res = dev.check(pk)
            _, orc = cref.check_history(hm.as_c(), model="mutex", threads=8)
            np.testing.assert_array_equal(res.valid, orc["valid"])
            np.testing.assert_array_equal(res.fail_event, orc["fail_event"])
            continue
        _, res, _ = device_vs_oracle(h, dev)
        if first is None:
            first = res
    again = dev.check(Packed(seq[0]))
    np.testing.assert_array_equal(again.valid, first.valid)
    np.testing.assert_array_equal(again.fail_event, first.fail_event)


def test_malformed_batch_rejected_then_context_reusable():
    """A batch whose event stream breaks the pairing invariants is refused with
    LC_E_INVALID and a message naming the key, and the same context then checks
    a good batch bit-exactly.  Every key of this batch fits the register tier,
    so the events are checked by T0 as it walks them (T0_STRICT), on both the
    host-to-host and the resident path."""
    import ctypes as C
    from lincheck import _native as N
    from lincheck.checker import Packed
    dev = Device(0)
    h = H.synth(n_keys=400, ops_per_key=200, concurrency=6, seed=41)
    pk = Packed(h)
    n_ev = int(pk.ev_off[-1])
    # the 32-bit words, when lc_pack gave them (ABI 11: only the 16-bit ones
    # when every word fits)
    ev = np.ctypeslib.as_array(pk.view.events, shape=(n_ev,)) if pk.view.events else None
    j = int(pk.ev_off[317])  # key 317's first event is an invoke: make it an :ok
    assert not pk.all_events()[j] & N.LC_EV_OK_BIT
    if ev is not None:
        saved = int(ev[j])
        ev[j] = saved | N.LC_EV_OK_BIT
    # the 16-bit copy the register tier is uploaded from (lc_batch.events16)
    ev16 = np.ctypeslib.as_array(pk.view.events16, shape=(n_ev,)) if pk.view.events16 else None
    if ev16 is not None:
        saved16 = int(ev16[j])
        ev16[j] = saved16 | 0x8000
    with pytest.raises(N.LincheckError) as ei:
        dev.check(pk)
    assert ei.value.code == -1 and "key 317" in str(ei.value)
    db = dev.upload(pk)  # T0 validates this batch: the upload takes it as it is
    with pytest.raises(N.LincheckError) as ei:
        db.check(peak=False)
    assert ei.value.code == -1 and "key 317" in str(ei.value)
    if ev is not None:
        ev[j] = saved
    if ev16 is not None:
        ev16[j] = saved16
    device_vs_oracle(h, dev)


def test_async_resident_steps():
    """LC_DEV_ASYNC: register-tier-only steps are only enqueued, lc_wait
    returns their count and span, and the verdicts equal a synchronous check's
    (and the oracle's).  A batch with keys beyond the register tier ignores
    the flag and runs synchronously (lc_wait then counts 0)."""
    import ctypes as C
    from lincheck import _native as N
    from lincheck.checker import Packed
    dev = Device(0)
    for h, t0_only in ((H.synth(n_keys=600, ops_per_key=700, concurrency=10, anomaly_rate=0.05, seed=51), True),
                       (H.synth(n_keys=16, ops_per_key=600, concurrency=16, seed=17), False)):
        pk = Packed(h)
        db = dev.upload(pk)
        K = pk.n_keys
        valid, fe, cause = _HipBuf(K), _HipBuf(4 * K), _HipBuf(K)
        for b in (valid, fe, cause):
            b.fill(0x5A)
        r = N.LcResult(C.cast(valid.ptr, N.P(C.c_int8)), C.cast(fe.ptr, N.P(C.c_int32)),
                       C.cast(cause.ptr, N.P(C.c_uint8)), None, None, None)
        dev.wait()
        for _ in range(4):
            st = db.check_into(r, asynchronous=True)
        dev.wait_step(1)  # lc_wait_step: the step before the latest (or everything)
        dev.wait_step(0)
        n, span = dev.wait()
        if t0_only:
            assert n == 4 and span > 0 and st.kernel_ms == 0
        else:
            assert n == 0 and st.kernel_ms > 0
        ref = db.check(peak=False)
        np.testing.assert_array_equal(valid.get(np.int8), ref.valid)
        np.testing.assert_array_equal(fe.get(np.int32), ref.fail_event)
        np.testing.assert_array_equal(cause.get(np.uint8), ref.cause)
        _, orc = cref.check_history(h.as_c(), budget=dev.budget, threads=8)
        np.testing.assert_array_equal(ref.valid, orc["valid"])
        np.testing.assert_array_equal(ref.fail_event, orc["fail_event"])


def test_wait_step_two_result_sets():
    """lc_wait_step(1) waits for the asynchronous step before the latest: with
    two result sets (the N > 1 bench's double buffer), set A is complete --
    read while step B may still run -- and equals the oracle; a synchronous
    step (a batch whose keys leave the register tier) between asynchronous
    ones does not shift which step that is; a `back` beyond the steps on
    record waits for everything."""
    import ctypes as C
    from lincheck import _native as N
    from lincheck.checker import Packed
    dev = Device(0)
    h = H.synth(n_keys=800, ops_per_key=700, concurrency=10, anomaly_rate=0.05, seed=53)
    pk = Packed(h)
    db = dev.upload(pk)
    K = pk.n_keys
    _, orc = cref.check_history(h.as_c(), budget=dev.budget, threads=8)
    h2 = H.synth(n_keys=16, ops_per_key=600, concurrency=16, seed=17)  # beyond T0: a synchronous step
    db2 = dev.upload(Packed(h2))

    def result_set():
        bufs = (_HipBuf(K), _HipBuf(4 * K), _HipBuf(K))
        for b in bufs:
            b.fill(0x5A)
        r = N.LcResult(C.cast(bufs[0].ptr, N.P(C.c_int8)), C.cast(bufs[1].ptr, N.P(C.c_int32)),
                       C.cast(bufs[2].ptr, N.P(C.c_uint8)), None, None, None)
        return bufs, r

    def assert_oracle(bufs):
        np.testing.assert_array_equal(bufs[0].get(np.int8), orc["valid"])
        np.testing.assert_array_equal(bufs[1].get(np.int32), orc["fail_event"])
        np.testing.assert_array_equal(bufs[2].get(np.uint8), orc["cause"])

    dev.wait()
    (a_bufs, ra), (b_bufs, rb) = result_set(), result_set()
    db.check_into(ra, asynchronous=True)
    db.check_into(rb, asynchronous=True)
    dev.wait_step(1)
    assert_oracle(a_bufs)
    dev.wait_step(0)
    assert_oracle(b_bufs)
    n, _ = dev.wait()
    assert n == 2

    (a_bufs, ra), (b_bufs, rb) = result_set(), result_set()
    db.check_into(ra, asynchronous=True)
    db2.check(peak=False)  # synchronous: not an asynchronous step on record
    db.check_into(rb, asynchronous=True)
    dev.wait_step(1)
    assert_oracle(a_bufs)
    dev.wait_step(7)  # no such step on record: everything
    assert_oracle(b_bufs)
    n, _ = dev.wait()
    assert n == 2


def test_concurrent_calls_on_one_context():
    """independent/checker calls its inner checker from a
    bounded pmap, so one context may be entered from several threads at once.
    Calls are serialised inside the library; every thread's verdicts must be
    its own batch's (bit-exact with the oracle)."""
    import threading
    from lincheck.checker import Packed
    dev = Device(0)
    hs = [H.synth(n_keys=n, ops_per_key=300, concurrency=8, anomaly_rate=0.1, seed=60 + i)
          for i, n in enumerate((300, 50, 700, 5, 260, 1000))]
    pks = [Packed(h) for h in hs]
    out, errs = [None] * len(hs), []

    def run(i):
        try:
            for _ in range(3):
                out[i] = dev.check(pks[i], verdicts_only=(i % 2 == 0))
        except Exception as e:  # noqa: BLE001 -- reported below
            errs.append(e)

    ts = [threading.Thread(target=run, args=(i,)) for i in range(len(hs))]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errs, errs
    for h, res in zip(hs, out):
        _, orc = cref.check_history(h.as_c(), budget=dev.budget, threads=8)
        np.testing.assert_array_equal(res.valid, orc["valid"])
        np.testing.assert_array_equal(res.fail_event, orc["fail_event"])


def _c5_bench_history():
    """bench.py --config C5: 1,000 keys x 1,000 ops, concurrency 10, 5 %
    anomalous keys, seed 5 (BASELINE configs[4])."""
    return H.synth(n_keys=1000, ops_per_key=1000, concurrency=10, anomaly_rate=0.05, seed=5)


def _c5_subhistories(h, keys):
    """Each key's sub-history (independent/subhistory: the key's rows, tuple
    values unwrapped), built from the history's own key column -- not from
    the packed batch, so the split is checked too."""
    kk = np.asarray(h.key)
    out = {}
    for k in keys:
        sub = []
        for r in np.flatnonzero(kk == k):
            o = h.op(int(r))
            v = o.get("value")
            if getattr(v, "_lc_tuple", False):
                o["value"] = v[1]
            sub.append(o)
        out[k] = sub
    return out


def test_c5_full_size_counterexamples_linear():
    """BASELINE config 5's "verdict plus counterexample
    parity" at its own size, through the Jepsen-shaped path at
    etcdemo.clj:115-119 (independent/checker over compose {:linear
    (linearizable {:model cas-register :algorithm :linear}), :timeline}) --
    the exact speculative segments (k_spec<..., EX>, final configs, no
    peaks).  Every key's :valid? equals the C restatement's; for every
    invalid key, :op / :previous-ok / :last-op :index, the :configs set and
    the :final-paths set equal oracle/linear_ref.py's analysis of the key's
    sub-history (subsets when the restatement has more than 10, jepsen's
    truncation)."""
    import linear_ref as LR
    from helpers import config_tuple, path_tuple
    from lincheck import checker as ck
    from lincheck import independent, model
    h = _c5_bench_history()
    lin = ck.linearizable({"model": model.cas_register(), "algorithm": "linear"})
    out = independent.checker(ck.compose({"linear": lin, "timeline": ck.unbridled_optimism()})).check({}, h, {})
    keys, orc = cref.check_history(h.as_c(), threads=8)
    exp_valid = {int(k): {1: True, 0: False, -1: "unknown"}[int(r["valid"])] for k, r in zip(keys, orc)}
    assert {k: r["linear"]["valid?"] for k, r in out["results"].items()} == exp_valid
    bad = sorted(k for k, v in exp_valid.items() if v is False)
    assert sorted(out["failures"]) == bad and out["valid?"] is False
    subs = _c5_subhistories(h, bad)
    n_cfg = n_paths = 0
    for k in bad:
        sub, m = subs[k], out["results"][k]["linear"]
        a = LR.analysis(sub)
        assert a.valid is False
        assert m["op"]["index"] == sub[a.fail_pos]["index"] and m["op"]["type"] == "ok", k
        prev = sub[a.previous_ok_pos]["index"] if a.previous_ok_pos is not None else None
        assert (m["previous-ok"] or {}).get("index") == prev, k
        assert (m["last-op"] or {}).get("index") == prev, k
        exp_cfgs = {(st, frozenset(sub[a.ops[q].invoke_pos]["index"] for q in L)) for st, L in a.final_configs}
        got_cfgs = [config_tuple(c, "cas-register") for c in m["configs"]]
        assert len(set(got_cfgs)) == len(got_cfgs) == min(10, len(exp_cfgs)), k
        assert set(got_cfgs) <= exp_cfgs, k
        if len(exp_cfgs) <= 10:
            assert set(got_cfgs) == exp_cfgs, k
        exp_paths = LR.final_paths(a, sub)
        got_paths = {path_tuple(p, "cas-register") for p in m["final-paths"]}
        assert len(got_paths) == len(m["final-paths"]) > 0, k
        assert exp_paths is not None and got_paths <= exp_paths, k
        if len(exp_cfgs) <= 10 and len(exp_paths) <= 10:
            assert got_paths == exp_paths, k
        n_cfg += len(got_cfgs)
        n_paths += len(got_paths)
    assert len(bad) > 20 and n_cfg >= len(bad) and n_paths >= len(bad)


def test_c5_full_size_counterexamples_wgl():
    """The same history through (linearizable {:algorithm :wgl}): every key's
    :valid? equals oracle/wgl_ref.c's; for every invalid key, :op and
    :previous-ok :index and the :configs frontier equal oracle/wgl_ref.py's
    walk on the key's sub-history (a subset when its frontier has more than
    10 configs)."""
    import wgl_ref as W
    from lincheck import checker as ck
    from lincheck import independent, model
    h = _c5_bench_history()
    lin = ck.linearizable({"model": model.cas_register(), "algorithm": "wgl"})
    out = independent.checker(lin).check({}, h, {})
    keys, orc, _, _ = cref.check_history_wgl(h.as_c(), threads=8)
    exp_valid = {int(k): {1: True, 0: False, -1: "unknown"}[int(r["valid"])] for k, r in zip(keys, orc)}
    assert {k: r["valid?"] for k, r in out["results"].items()} == exp_valid
    bad = sorted(k for k, v in exp_valid.items() if v is False)
    assert sorted(out["failures"]) == bad
    subs = _c5_subhistories(h, bad)
    n_cfg = 0
    for k in bad:
        sub, g = subs[k], out["results"][k]
        w = W.analysis(sub)
        assert w.valid is False and g["analyzer"] == "wgl"
        assert g["op"]["index"] == sub[w.fail_pos]["index"], k
        prev = sub[w.previous_ok_pos]["index"] if w.previous_ok_pos is not None else None
        assert (g["previous-ok"] or {}).get("index") == prev, k
        idx = lambda oid: sub[w.ops[oid].invoke_pos]["index"]
        want = {(st, frozenset(idx(q) for q in L)) for st, L in w.frontier}
        got = {(c["model"]["value"], frozenset(o["index"] for o in c["linearized"])) for c in g["configs"]}
        assert got and got <= want, k
        if len(want) <= 10:
            assert got == want, k
        n_cfg += len(got)
    assert len(bad) > 20 and n_cfg >= len(bad)
