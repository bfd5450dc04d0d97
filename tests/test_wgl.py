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
