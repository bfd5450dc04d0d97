"""Host side of the Checker mirror (jepsen.checker / jepsen.independent,
etcdemo.clj:115-119, :165-167) without a GPU: result merging, check-safe,
and the Knossos-shaped result maps built from per-key verdict records."""
import json
import os

import numpy as np
import pytest

import cref
from lincheck import checker as ck
from lincheck import history as H
from lincheck import independent, model
from lincheck.checker import KeyResults, Packed, _render_key
from lincheck.independent import Tuple

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "kat.json")


def test_merge_valid():
    assert ck.merge_valid([True, True]) is True
    assert ck.merge_valid([True, "unknown"]) == "unknown"
    assert ck.merge_valid(["unknown", False, True]) is False
    assert ck.merge_valid([]) is True


class Boom:
    def check(self, test, history, opts):
        raise RuntimeError("boom")


class Const:
    def __init__(self, v):
        self.v = v

    def check(self, test, history, opts):
        return {"valid?": self.v, "n": len(history)}


def test_check_safe_turns_exceptions_into_unknown():
    r = ck.check_safe(Boom(), {}, [], {})
    assert r["valid?"] == "unknown" and "boom" in r["error"]


def test_compose():
    r = ck.compose({"a": Const(True), "b": Boom()}).check({}, [], {})
    assert r["valid?"] == "unknown" and r["a"]["valid?"] is True


def test_independent_checker_generic_inner():
    ops = [{"type": "invoke", "f": "read", "value": Tuple(k, None), "process": k} for k in range(3)]
    ops.append({"type": "info", "f": "start", "value": None, "process": "nemesis"})
    verdicts = {0: True, 1: False, 2: "unknown"}

    class PerKey:
        def check(self, test, history, opts):
            k = opts["history-key"]
            assert all((not independent.is_tuple(o["value"])) for o in history)
            assert history[-1]["process"] == "nemesis"  # non-tuple ops stay in every sub-history
            return {"valid?": verdicts[k]}

    r = independent.checker(PerKey()).check({}, ops, {})
    assert r["valid?"] is False
    assert r["failures"] == [1]  # :unknown is truthy in Clojure, so not a failure
    assert set(r["results"]) == {0, 1, 2}


def test_linearizable_options():
    with pytest.raises(ValueError):
        ck.linearizable({})
    # F-3: :wgl and the default (competition) run the same device search
    assert ck.linearizable({"model": model.cas_register(), "algorithm": "wgl"}).analyzer == "wgl"
    comp = ck.linearizable({"model": model.cas_register()})
    assert comp.algorithm == 2 and comp.analyzer == "linear"
    lin = ck.linearizable({"model": model.cas_register(), "algorithm": "linear"})
    assert ck.batched_linearizable(lin) is lin
    comp = ck.compose({"linear": lin, "timeline": ck.unbridled_optimism()})
    assert ck.batched_linearizable(comp) is lin


def test_other_model_messages():
    m = model.mutex()
    assert m.step("acquire").locked is True
    assert m.step("release").msg == "not held"
    assert m.step("acquire").step("acquire").msg == "already held"
    r = model.register()
    assert r.step("write", 3).step("read", 1).msg == "3≠1"
    with pytest.raises(ValueError):
        r.step("cas", [1, 2])


def test_model_messages():
    r = model.cas_register()
    assert r.step("write", 3).value == 3
    assert r.step("cas", [3, 4]).msg == "can't CAS nil from 3 to 4"
    assert r.step("write", 3).step("read", 1).msg == "can't read 1 from register 3"
    assert r.step("write", 2).step("read", None).value == 2


def kats():
    cases = json.load(open(GOLDEN))
    for c in cases:
        for op in c["history"]:
            v = op["value"]
            if isinstance(v, dict) and "tuple" in v:
                op["value"] = Tuple(*v["tuple"])
    return cases


@pytest.mark.parametrize("case", kats(), ids=lambda c: c["name"])
def test_result_maps_from_verdict_records(case):
    """Knossos-shaped maps (A8) from verdict records: :op / :previous-ok are
    the original op maps (their :index), :configs render the model value."""
    h = H.History.from_ops(case["history"])
    mdl = {"cas-register": model.cas_register(), "register": model.register(),
           "mutex": model.mutex()}[case.get("model", "cas-register")]
    pk = Packed(h, mdl)
    keys, r = cref.check_history(h.as_c(), model=mdl.name)
    K = pk.n_keys
    res = KeyResults(r["valid"], r["fail_event"], r["cause"], r["peak"],
                     np.zeros((K, 10, 2), np.uint64), np.zeros(K, np.uint32), {})
    for i, k in enumerate(pk.keys):
        m = _render_key(pk, i, res, None)
        exp = case["expect"][str(k)]
        assert m["valid?"] == exp["valid?"]
        if exp["valid?"] == "unknown":  # check-safe: {:valid? :unknown :error ...}
            assert m["error"] and set(m) == {"valid?", "error"}
            continue
        assert m["analyzer"] == "linear"
        if not exp["valid?"]:
            assert m["op"]["index"] == exp["op"]
            assert m["op"]["type"] == "ok"
            assert m["previous-ok"]["index"] == exp["previous-ok"]


def _final_paths_case(ops, model_name):
    """Render :configs / :final-paths from the restatement's final configs and
    compare them with the restatement's own enumeration."""
    import linear_ref as LR
    from helpers import config_tuple, encode_finals, path_tuple
    mdl = {"cas-register": model.cas_register(), "register": model.register(),
           "mutex": model.mutex()}[model_name]
    h = H.History.from_ops(ops)
    pk = Packed(h, mdl)
    checked = 0
    for i, k in enumerate(pk.keys):
        sub = LR.subhistory(ops, k)
        a = LR.analysis_safe(sub, model=model_name)
        if a.valid is not False:
            continue
        fin, n = encode_finals(pk, i, a, model_name)
        K = pk.n_keys
        final = np.zeros((K, 10, 2), np.uint64); final[i] = fin
        nf = np.zeros(K, np.uint32); nf[i] = n
        valid = np.ones(K, np.int8); valid[i] = 0
        fev = np.full(K, -1, np.int32); fev[i] = a.fail_event
        res = KeyResults(valid, fev, np.zeros(K, np.uint8), np.zeros(K, np.uint32), final, nf, {})
        m = _render_key(pk, i, res, None)
        exp_paths = LR.final_paths(a, sub, model_name)
        got = [path_tuple(p, model_name) for p in m["final-paths"]]
        assert len(set(got)) == len(got)
        assert set(got) <= exp_paths
        if len(exp_paths) <= 10 and len(a.final_configs) <= 10:
            assert set(got) == exp_paths
        else:
            assert len(got) == 10
        # every path replays under the host model: legal steps, then the failure
        for p in m["final-paths"]:
            st = mdl.of_state(None)
            st = type(mdl)(**{f: v for f, v in zip(p[0]["model"].keys(), p[0]["model"].values())}) \
                if model_name != "mutex" else model.Mutex(p[0]["model"]["locked?"])
            for e in p[1:-1]:
                st = st.step(e["op"]["f"], e["op"]["value"])
                assert not isinstance(st, model.Inconsistent)
                assert st.render() == e["model"]
            bad = st.step(p[-1]["op"]["f"], p[-1]["op"]["value"])
            assert isinstance(bad, model.Inconsistent) and bad.msg == p[-1]["model"]["msg"]
        cfgs = {config_tuple(c, model_name) for c in m["configs"]}
        exp_cfgs = {(oracle_v(st, model_name), frozenset(sub[a.ops[q].invoke_pos]["index"] for q in L))
                    for st, L in a.final_configs[:10]}
        assert cfgs == exp_cfgs
        checked += 1
    return checked


def oracle_v(st, model_name):
    return bool(st) if model_name == "mutex" else st


@pytest.mark.parametrize("case", kats(), ids=lambda c: c["name"])
def test_final_paths_known_answers(case):
    """:final-paths / :configs on the known answers."""
    _final_paths_case(case["history"], case.get("model", "cas-register"))


@pytest.mark.parametrize("model_name", ["cas-register", "register", "mutex"])
def test_final_paths_random(model_name):
    from histgen import random_history
    checked = 0
    for seed in range(400):
        ops = random_history(seed, n_keys=2, max_ops=8, procs=4, model=model_name)
        checked += _final_paths_case(ops, model_name)
    assert checked > 20


@pytest.mark.parametrize("inner_kind", ["linearizable", "compose"])
def test_fast_result_shaping_equals_general(inner_kind):
    """Linearizable._shape_fast (shared maps for the valid keys, merge-valid
    from the verdict array) returns what the general per-key shaping does,
    on a C5-shaped batch whose device results are stood in by the C
    restatement's (no GPU here: verdicts, causes, failing events; one key
    made :unknown at the budget)."""
    import cref
    from lincheck import _native as N
    h = H.synth(n_keys=300, ops_per_key=200, concurrency=8, anomaly_rate=0.1, seed=12)
    keys, orc = cref.check_history(h.as_c(), threads=4)
    K = len(keys)
    valid = orc["valid"].astype(np.int8).copy()
    cause = orc["cause"].astype(np.uint8).copy()
    valid[5], cause[5] = -1, 2  # :unknown at the budget
    res = KeyResults(valid=valid, fail_event=orc["fail_event"].astype(np.int32), cause=cause,
                     peak=np.zeros(K, np.uint32), final=np.zeros((K, 10, 2), np.uint64),
                     n_final=np.zeros(K, np.uint32), stats={"kernel_ms": 0.0})

    class FakeDev:
        def check(self, packed, peaks=True, verdicts_only=False):
            return res

    outs = []
    for fast in (True, False):
        lin = ck.linearizable({"model": model.cas_register(), "algorithm": "linear"})
        lin._dev = lambda: FakeDev()
        inner = lin if inner_kind == "linearizable" else ck.compose({"linear": lin,
                                                                     "timeline": ck.unbridled_optimism()})
        old = ck.SHARED_VALID_MAPS
        ck.SHARED_VALID_MAPS = fast
        try:
            outs.append(independent.checker(inner).check({}, h, {}))
        finally:
            ck.SHARED_VALID_MAPS = old
    a, b = outs
    assert list(a["results"]) == list(b["results"]) == [int(k) for k in keys]
    assert a["results"] == b["results"]
    assert a["failures"] == b["failures"] and a["failures"]
    assert a["valid?"] == b["valid?"] is False
