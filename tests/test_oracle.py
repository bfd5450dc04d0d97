"""The oracle is pinned before it is trusted: the Python restatement of
knossos.linear, the definitional brute-force checker and the C restatement
must agree with the hand-derived known answers (tests/golden/kat.json) and
with each other on random and synthetic histories."""
import json
import os

import numpy as np
import pytest
from hypothesis import given, settings, strategies as st

import brute
import cref
import linear_ref as LR
from histgen import random_history
from lincheck import history as H
from lincheck.independent import Tuple

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "kat.json")
CAUSE = {"none": 0, "nonlin": 1, "budget": 2, "window": 3, "states": 4, "error": 5}


def load_kats():
    with open(GOLDEN) as f:
        cases = json.load(f)
    for c in cases:
        for op in c["history"]:
            v = op["value"]
            if isinstance(v, dict) and "tuple" in v:
                op["value"] = Tuple(*v["tuple"])
    return cases


@pytest.mark.parametrize("case", load_kats(), ids=lambda c: c["name"])
def test_known_answers(case):
    ops = case["history"]
    model = case.get("model", "cas-register")
    # Python restatement + brute force
    for k in LR.history_keys(ops):
        sub = LR.subhistory(ops, k)
        exp = case["expect"][str(k)]
        a = LR.analysis_safe(sub, model=model)
        assert a.valid == exp["valid?"]
        if exp["valid?"] == "unknown":  # check-safe around one key
            assert a.cause == "error"
            continue
        assert brute.brute_check(sub, model=model)[0] == exp["valid?"]
        if not exp["valid?"]:
            assert sub[a.fail_pos]["index"] == exp["op"]
            assert sub[a.previous_ok_pos]["index"] == exp["previous-ok"]
    # C restatement
    h = H.History.from_ops(ops)
    keys, r = cref.check_history(h.as_c(), model=model)
    for k, rr in zip(keys, r):
        exp = case["expect"][str(k)]
        assert rr["valid"] == {True: 1, False: 0, "unknown": -1}[exp["valid?"]]
        if exp["valid?"] == "unknown":
            assert rr["cause"] == 5 and rr["fail_event"] == -1


@settings(max_examples=300, deadline=None)
@given(st.integers(0, 2**31 - 1))
def test_restatement_matches_brute_force(seed):
    ops = random_history(seed)
    for k in LR.history_keys(ops):
        sub = LR.subhistory(ops, k)
        a = LR.analysis(sub)
        ok, fe = brute.brute_check(sub)
        assert a.valid == ok
        assert a.fail_event == fe


def py_vs_c(ops, budget):
    h = H.History.from_ops(ops)
    keys, r = cref.check_history(h.as_c(), budget=budget, threads=2)
    assert list(keys) == LR.history_keys(ops)
    for k, rr in zip(keys, r):
        a = LR.analysis(LR.subhistory(ops, k), budget=budget)
        v = {True: 1, False: 0, "unknown": -1}[a.valid]
        assert rr["valid"] == v
        assert rr["cause"] == CAUSE[a.cause]
        assert rr["fail_event"] == (-1 if a.fail_event is None else a.fail_event)
        if a.cause != "budget":
            assert rr["peak"] == a.peak_configs
            assert rr["probes"] == a.probes


@settings(max_examples=200, deadline=None)
@given(st.integers(0, 2**31 - 1), st.sampled_from([1 << 20, 3, 6]))
def test_c_restatement_matches_python(seed, budget):
    py_vs_c(random_history(seed, n_keys=3, max_ops=9, procs=4), budget)


@pytest.mark.parametrize("kw", [
    dict(n_keys=4, ops_per_key=150, concurrency=5, seed=3),
    dict(n_keys=3, ops_per_key=200, concurrency=8, anomaly_rate=1.0, seed=5),
    dict(n_keys=2, ops_per_key=120, concurrency=6, info_rate=0.05, seed=4),
    dict(n_keys=3, ops_per_key=60, concurrency=5, interleave=True, nemesis_period=3.0, seed=1),
])
def test_c_restatement_matches_python_on_synthetic(kw):
    py_vs_c(H.synth(**kw).to_ops(), 1 << 14)


def test_budget_semantics_exact():
    """With a budget just below / at a key's peak the verdict flips to
    :unknown exactly at the event where the set first exceeds it."""
    ops = H.synth(n_keys=1, ops_per_key=120, concurrency=6, seed=9).to_ops()
    a = LR.analysis(LR.subhistory(ops, 0))
    assert a.valid is True
    peak = a.peak_configs
    assert LR.analysis(LR.subhistory(ops, 0), budget=peak - 1).valid == "unknown"
    # closure may exceed the final set: find the smallest budget that passes
    b = peak
    while LR.analysis(LR.subhistory(ops, 0), budget=b).valid != True:  # noqa: E712
        b += 1
    keys, r = cref.check_history(H.History.from_ops(ops).as_c(), budget=b)
    assert r["valid"][0] == 1
    keys, r = cref.check_history(H.History.from_ops(ops).as_c(), budget=b - 1)
    assert r["valid"][0] == -1


@settings(max_examples=200, deadline=None)
@given(st.integers(0, 2**31 - 1), st.sampled_from(["mutex", "register"]))
def test_other_models_restatement_matches_brute_force(seed, model):
    """(model/mutex), (model/register): JIT restatement =
    definition, and the C restatement agrees with the Python one."""
    ops = random_history(seed, model=model)
    for k in LR.history_keys(ops):
        sub = LR.subhistory(ops, k)
        a = LR.analysis(sub, model=model)
        ok, fe = brute.brute_check(sub, model=model)
        assert a.valid == ok
        assert a.fail_event == fe
    h = H.History.from_ops(ops)
    keys, r = cref.check_history(h.as_c(), model=model)
    for k, rr in zip(keys, r):
        a = LR.analysis(LR.subhistory(ops, k), model=model)
        assert rr["valid"] == {True: 1, False: 0, "unknown": -1}[a.valid]
        assert rr["fail_event"] == (-1 if a.fail_event is None else a.fail_event)
        assert rr["peak"] == a.peak_configs and rr["probes"] == a.probes
