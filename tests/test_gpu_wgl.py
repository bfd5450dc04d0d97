"""knossos.wgl on the device (LC_ALGO_WGL, device_wgl.hip; the :algorithm slot
at etcdemo.clj:118) against the C restatement
(oracle/wgl_ref.c, itself checked against oracle/wgl_ref.py in
tests/test_wgl.py): per key the verdict, cause, failing event, Lowe's cache
size at the end (the budget is a cache-size bound, so an :unknown is only
reproducible if the walk is the same walk) and the frontier records (the
first max_final the walk reaches, as {slot mask, state}) are bit-identical.
Parity with Knossos itself is unpinned."""
import numpy as np
import pytest

import cref
import linear_ref as LR
import wgl_ref as W
from histgen import random_history
from lincheck import _native as N
from lincheck import checker as ck
from lincheck import history as H
from lincheck import independent, model
from lincheck.checker import Device, Packed

pytestmark = pytest.mark.gpu

NIL = -(1 << 63)


def wgl_vs_oracle(hist: H.History, budget: int, model_name: str = "cas-register", path_flags: int = 0):
    mdl = {"cas-register": model.cas_register, "register": model.register, "mutex": model.mutex}[model_name]()
    packed = Packed(hist, mdl)
    dev = Device(0, budget=budget, algorithm=N.LC_ALGO_WGL, path_flags=path_flags)
    res = dev.check(packed)
    keys, orc, fin, nf = cref.check_history_wgl(hist.as_c(), budget=budget, threads=8, model=model_name)
    assert list(keys) == packed.keys
    np.testing.assert_array_equal(res.valid, orc["valid"], err_msg="valid?")
    np.testing.assert_array_equal(res.cause, orc["cause"], err_msg="cause")
    np.testing.assert_array_equal(res.fail_event, orc["fail_event"], err_msg="fail event")
    done = np.isin(orc["cause"], [0, 1, 2])
    np.testing.assert_array_equal(res.peak[done], orc["peak"][done], err_msg="cache size")
    assert (res.analyzer == N.LC_ALGO_WGL).all()
    bad = np.nonzero(orc["valid"] == 0)[0]
    np.testing.assert_array_equal(res.n_final[bad], nf[bad], err_msg="frontier size")
    for i in bad:
        for j in range(int(nf[i])):
            lo, hi = (int(x) for x in res.final[i, j])
            st = (hi >> 48) & 0x7FFF
            v = packed.state_value(int(i), st)
            want_v = None if int(fin[i, j, 2]) == NIL else int(fin[i, j, 2])
            if model_name == "mutex":
                v = 1 if v else None  # lc_pack interns locked as 1
            assert v == want_v, (i, j)
            assert lo == int(fin[i, j, 0]) & (2**64 - 1), (i, j)
            assert hi & ((1 << 48) - 1) == int(fin[i, j, 1]) & ((1 << 48) - 1), (i, j)
    return packed, res, orc


@pytest.mark.parametrize("seed", range(6))
def test_wgl_random_histories(seed):
    """Small multi-key histories: crashes, failures, unmatched invocations,
    nemesis ops, garbage reads; generous and tiny budgets."""
    ops = random_history(7000 + seed, n_keys=40, max_ops=24, procs=5, p_info=0.08, p_garbage_read=0.15)
    h = H.History.from_ops(ops)
    for budget in (1 << 20, 5, 40):
        wgl_vs_oracle(h, budget)


@pytest.mark.parametrize("model_name", ["register", "mutex"])
def test_wgl_other_models(model_name):
    ops = random_history(91, n_keys=60, max_ops=16, procs=4, p_info=0.05, model=model_name)
    wgl_vs_oracle(H.History.from_ops(ops), 1 << 20, model_name)


@pytest.mark.parametrize("name,kw,budget", [
    ("c2", dict(n_keys=300, ops_per_key=1000, concurrency=10, seed=2), 1 << 20),
    ("c5", dict(n_keys=300, ops_per_key=1000, concurrency=10, anomaly_rate=0.1, seed=5), 1 << 20),
    ("c1", dict(n_keys=6, ops_per_key=100, concurrency=10, interleave=True, nemesis_period=5.0, seed=1,
                anomaly_rate=0.5), 1 << 20),
])
def test_wgl_config_shapes(name, kw, budget):
    _, res, orc = wgl_vs_oracle(H.synth(**kw), budget)
    if name == "c5":
        assert (orc["valid"] == 0).sum() > 5


def test_wgl_c4_shaped_keys_decided():
    """VERDICT r3's C4-shaped keys (30 clients, 2 % crashed write/cas, seed
    4, budget 2^16; 4 keys each at 300, 600 and 1,200 ops): :linear gives up
    on every one at the budget, the device's WGL decides the ones its own
    restatement decides, and gives up on the same others."""
    decided = 0
    for n in (300, 600, 1200):
        h = H.synth(n_keys=4, ops_per_key=n, concurrency=30, info_rate=0.02, seed=4)
        _, res, orc = wgl_vs_oracle(h, 1 << 16)
        decided += int((res.valid != -1).sum())
    assert decided >= 7


def test_wgl_c4_full_size():
    """C4 exactly as bench.py runs it (256 keys x 5,000 ops, 30 clients, 2 %
    crashed, budget 2^16): every key's walk, to its cache size, equals the
    restatement's."""
    wgl_vs_oracle(H.synth(n_keys=256, ops_per_key=5000, concurrency=30, info_rate=0.02, seed=4), 1 << 16)


def test_wgl_spill_to_budget_tables():
    """Keys whose cache outgrows the shared tables (LC_PATH_WGL_SMALL: 2^14
    entries) are searched again with a table the budget fits: the same
    records, and the step reports them."""
    h = H.synth(n_keys=8, ops_per_key=600, concurrency=30, info_rate=0.02, seed=4)
    _, res, _ = wgl_vs_oracle(h, 1 << 16, path_flags=N.LC_PATH_WGL_SMALL)
    assert res.stats["wgl_spilled"] > 0


def test_wgl_window_limit_on_device():
    ops = []
    for p in range(115):
        ops.append({"type": "invoke", "f": "write", "value": independent.Tuple(0, 1), "process": p})
        ops.append({"type": "info", "f": "write", "value": independent.Tuple(0, 1), "process": p})
    ops.append({"type": "invoke", "f": "read", "value": independent.Tuple(1, None), "process": 500})
    ops.append({"type": "ok", "f": "read", "value": independent.Tuple(1, 3), "process": 500})
    for i, o in enumerate(ops):
        o["index"] = i
    _, res, orc = wgl_vs_oracle(H.History.from_ops(ops), 1 << 20)
    assert list(res.cause) == [3, 1]


def test_competition_answers_budget_keys_with_wgl():
    """The default :algorithm (knossos.competition): :linear's answer where
    it has one, WGL's (with :analyzer :wgl) for the keys :linear gives up on
    at the budget -- on C4-shaped keys, WGL's restatement's verdicts."""
    budget = 1 << 16
    h = H.synth(n_keys=4, ops_per_key=300, concurrency=30, info_rate=0.02, seed=4)
    ops = h.to_ops()
    lin = ck.linearizable({"model": model.cas_register(), "max-configs": budget})
    out = independent.checker(lin).check({}, ops, {})
    for k, r in out["results"].items():
        w = W.analysis(LR.subhistory(ops, k), budget=budget)
        a = LR.analysis(LR.subhistory(ops, k), budget=budget)
        if a.valid == "unknown" and a.cause == "budget":
            assert r["analyzer"] == "wgl" and r["valid?"] == w.valid, k
        else:
            assert r["analyzer"] == "linear" and r["valid?"] == a.valid, k
    assert any(r["analyzer"] == "wgl" and r["valid?"] is True for r in out["results"].values())


@pytest.mark.parametrize("name,kw,budget", [
    ("c2", dict(n_keys=60, ops_per_key=1000, concurrency=10, seed=2), 1 << 20),
    ("c5", dict(n_keys=120, ops_per_key=1000, concurrency=10, anomaly_rate=0.2, seed=5), 1 << 20),
    ("c4", dict(n_keys=8, ops_per_key=1200, concurrency=30, info_rate=0.02, seed=4), 1 << 16),
])
def test_wgl_events_from_hbm(name, kw, budget):
    """the walk that reads a key's events, slot history and
    descriptors from HBM (wgl_key<false, *>: keys longer than the LDS
    staging) -- every key forced onto it (LC_PATH_WGL_EV_HBM), narrow and
    wide windows, valid, invalid and budget keys -- gives the restatement's
    records."""
    _, res, orc = wgl_vs_oracle(H.synth(**kw), budget, path_flags=N.LC_PATH_WGL_EV_HBM)
    if name == "c5":
        assert (orc["valid"] == 0).sum() > 5
    # Lowe's cache lookups (one per legal candidate of a probe round): every
    # pair the cache holds was a lookup's miss first
    assert res.stats["probes"] >= int(res.peak.astype(np.int64).sum())


def test_wgl_decides_c4_keys_at_a_larger_budget():
    """BASELINE C4's first 16 keys at full size (5,000 ops, 30 clients, 2 %
    crashed) at a cache budget of 2^20: :linear gives up on all of them at
    any budget measured (profiles/r05_c4_budget_sweep.json); the walk
    decides most, with the restatement's records, cache sizes included."""
    h = H.synth(n_keys=16, ops_per_key=5000, concurrency=30, info_rate=0.02, seed=4)
    _, res, orc = wgl_vs_oracle(h, 1 << 20)
    assert int((res.valid == 1).sum()) >= 8
