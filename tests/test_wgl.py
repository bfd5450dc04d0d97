"""The WGL restatement (oracle/wgl_ref.py: Wing & Gong with Lowe's cache,
knossos.wgl's algorithm) against the definitional
brute-force checker, the linear restatement and the hand KATs.

WGL is a different search from knossos.linear's config sets (a backtracking
walk over a linked list of call / return entries), so it pins what the two
must share: the verdict, the :ok it is stuck on at its deepest (the first
whose prefix cannot be linearized), :previous-ok, and its frontier there,
which must equal the closure of linear's config set standing before that
:ok under the other pending ops.  Parity with Knossos itself is unpinned
(no JVM, no fixtures)."""
import json
import os

import pytest
from hypothesis import given, settings, strategies as st

import brute
import linear_ref as LR
import wgl_ref as W
from histgen import mutex_history, random_history
from lincheck.independent import Tuple

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "kat.json")


def _same(sub, model="cas-register"):
    w = W.analysis(sub, model=model)
    a = LR.analysis(sub, model=model)
    assert w.valid == a.valid
    if a.valid is False:
        assert w.fail_pos == a.fail_pos and w.op_id == a.op_id
        assert w.previous_ok_pos == a.previous_ok_pos
        assert w.frontier == W.closure(a, model)
    return w, a


@settings(max_examples=400, deadline=None)
@given(st.integers(0, 2**31 - 1))
def test_wgl_matches_brute_force_and_linear(seed):
    ops = random_history(seed, n_keys=2, max_ops=8, procs=4)
    for k in LR.history_keys(ops):
        sub = LR.subhistory(ops, k)
        w, a = _same(sub)
        ok, fe = brute.brute_check(sub)
        assert w.valid == ok


@settings(max_examples=150, deadline=None)
@given(st.integers(0, 2**31 - 1), st.sampled_from(["register", "mutex", "multi-register"]))
def test_wgl_other_models(seed, model):
    ops = random_history(seed, n_keys=2, max_ops=7, procs=3, model=model)
    for k in LR.history_keys(ops):
        _same(LR.subhistory(ops, k), model)


@pytest.mark.parametrize("seed", range(6))
def test_wgl_longer_histories(seed):
    """Longer keys (20-40 ops, 5 processes, crashes): frontiers of dozens of
    configs, still the closure of linear's set."""
    ops = random_history(1000 + seed, n_keys=3, max_ops=40, procs=5, p_info=0.05, p_garbage_read=0.1)
    bad = 0
    for k in LR.history_keys(ops):
        w, _ = _same(LR.subhistory(ops, k))
        bad += w.valid is False
    ops = mutex_history(seed, n_keys=5, rounds=20, corrupt=0.5)
    for k in LR.history_keys(ops):
        _same(LR.subhistory(ops, k), "mutex")


def test_wgl_known_answers():
    cases = json.load(open(GOLDEN))
    n = 0
    for case in cases:
        ops = case["history"]
        for op in ops:
            v = op.get("value")
            if isinstance(v, dict) and "tuple" in v:
                op["value"] = Tuple(*v["tuple"])
        model = case.get("model", "cas-register")
        for k in LR.history_keys(ops):
            exp = case["expect"][str(k)]
            sub = LR.subhistory(ops, k)
            try:
                w = W.analysis(sub, model=model)
            except LR.HistoryError:
                assert exp["valid?"] == "unknown"
                continue
            assert w.valid == exp["valid?"], case["name"]
            if exp["valid?"] is False:
                assert sub[w.fail_pos]["index"] == exp["op"]
                assert sub[w.previous_ok_pos]["index"] == exp["previous-ok"]
            n += 1
    assert n > 20


def test_wgl_budget():
    ops = random_history(7, n_keys=1, max_ops=30, procs=6, p_info=0.3)
    sub = LR.subhistory(ops, LR.history_keys(ops)[0])
    assert W.analysis(sub, budget=3).valid in ("unknown", True, False)
    assert W.analysis(sub, budget=1).valid == "unknown"


# ---- the C restatement (oracle/wgl_ref.c) against the Python one ------------
import numpy as np  # noqa: E402

import cref  # noqa: E402
from lincheck import history as H  # noqa: E402

CAUSE = {"none": 0, "nonlin": 1, "budget": 2, "window": 3, "states": 4, "error": 5}


def _slots(events):
    """Window slot of every op (lowest free at :invoke, freed at :ok), as
    lc_pack and wgl_ref.c assign them."""
    free, slot = list(range(128)), {}
    for kind, oid, _ in events:
        if kind == "invoke":
            slot[oid] = min(free)
            free.remove(slot[oid])
        else:
            free.append(slot[oid])
    return slot


def c_vs_python(ops, budget, model="cas-register"):
    """Per key: verdict, cause, failing event, cache size and frontier of
    wgl_ref.c equal to wgl_ref.py's (the C frontier is the first 10 the walk
    reaches: a subset of the Python set, all of it when that has <= 10)."""
    h = H.History.from_ops(ops)
    keys, r, fin, nf = cref.check_history_wgl(h.as_c(), budget=budget, threads=2, model=model)
    assert list(keys) == LR.history_keys(ops)
    out = []
    for i, k in enumerate(keys):
        sub = LR.subhistory(ops, k)
        try:
            w = W.analysis(sub, budget=budget, model=model)
        except LR.HistoryError:
            assert r["valid"][i] == -1 and r["cause"][i] == CAUSE["error"]
            continue
        assert r["valid"][i] == {True: 1, False: 0, "unknown": -1}[w.valid], (k, w.valid, w.cause)
        assert r["cause"][i] == CAUSE[w.cause], (k, w.cause)
        ops_k, events = LR.complete(sub, model)
        if w.cause in ("none", "nonlin"):
            assert r["peak"][i] == w.cache_size, (k, r["peak"][i], w.cache_size)
        if w.valid is False:
            assert events[r["fail_event"][i]][2] == w.fail_pos
            slot = _slots(events)
            want = set()
            for st_, lin in w.frontier:
                m = 0
                for q in lin:
                    m |= 1 << slot[q]
                val = (1 if st_ else None) if model == "mutex" else st_
                want.add((m, val))
            got = set()
            for j in range(nf[i]):
                lo, hi, val = (int(x) for x in fin[i, j])
                got.add(((lo & (2**64 - 1)) | ((hi & (2**64 - 1)) << 64), None if val == -(1 << 63) else val))
            assert nf[i] == min(10, len(want)) and len(got) == nf[i], (k, nf[i], len(want))
            assert got <= want
        out.append((k, w))
    return out


@settings(max_examples=200, deadline=None)
@given(st.integers(0, 2**31 - 1), st.sampled_from([1 << 20, 3, 7]),
       st.sampled_from(["cas-register", "register", "mutex"]))
def test_c_wgl_matches_python(seed, budget, model):
    c_vs_python(random_history(seed, n_keys=3, max_ops=12, procs=4, p_info=0.1, model=model), budget, model)


@pytest.mark.parametrize("kw", [
    dict(n_keys=3, ops_per_key=200, concurrency=8, anomaly_rate=1.0, seed=5),
    dict(n_keys=2, ops_per_key=120, concurrency=6, info_rate=0.05, seed=4),
    dict(n_keys=3, ops_per_key=60, concurrency=5, interleave=True, nemesis_period=3.0, seed=1),
])
def test_c_wgl_matches_python_on_synthetic(kw):
    c_vs_python(H.synth(**kw).to_ops(), 1 << 14)


def test_c_wgl_c4_shaped_keys():
    """VERDICT r3's C4-shaped keys (30 clients, 2 % crashed write/cas, seed 4,
    budget 2^16), the 300-op ones: :linear gives up on every key at the
    budget, WGL's walk decides most of them; C and Python agree step for
    step (same verdicts, same cache sizes)."""
    h = H.synth(n_keys=4, ops_per_key=300, concurrency=30, info_rate=0.02, seed=4)
    res = c_vs_python(h.to_ops(), 1 << 16)
    _, lin = cref.check_history(h.as_c(), budget=1 << 16, threads=4)
    assert (lin["valid"] == -1).all()
    assert sum(w.valid is True for _, w in res) >= 3


def test_wgl_window_limit():
    """More than 112 ops pending at once (crashed writes pile up): :unknown
    "window" before any search, in both restatements, at the same :invoke."""
    ops = []
    for p in range(115):
        ops.append({"type": "invoke", "f": "write", "value": Tuple(0, 1), "process": p, "index": len(ops)})
        ops.append({"type": "info", "f": "write", "value": Tuple(0, 1), "process": p, "index": len(ops)})
    w = W.analysis(LR.subhistory(ops, 0))
    assert w.valid == "unknown" and w.cause == "window"
    _, r, _, _ = cref.check_history_wgl(H.History.from_ops(ops).as_c())
    assert r["valid"][0] == -1 and r["cause"][0] == CAUSE["window"] and r["fail_event"][0] == 112
