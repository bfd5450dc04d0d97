"""BASELINE.json's configs and the hand known answers, through the HIP path.

* Every tests/golden/kat.json case goes through the demo's checker expression
  (etcdemo.clj:115-119: independent/checker over compose {:linear
  linearizable, :timeline ...}) on the device; :valid?, :failures and, for
  invalid keys, the :index of :op and :previous-ok must be the hand-derived
  expectation.
* C1 (configs[0], the demo re-check): history.edn on disk -> lc_edn_read ->
  device, per-key verdicts, causes and failing events equal to the oracle on
  the same file.
* C4 (configs[3]) at full size and the bench's budget: 256 keys x 5,000 ops,
  concurrency 30, 2 % crashed write/cas, bit-exact against the oracle.
"""
import json
import os

import numpy as np
import pytest

import cref
import linear_ref as LR
import wgl_ref as W
from helpers import device_vs_oracle
from histgen import random_history
from lincheck import checker as ck
from lincheck import history as H
from lincheck import independent, model
from lincheck.checker import Device, Packed
from lincheck.independent import Tuple

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "kat.json")
MODELS = {"cas-register": model.cas_register, "register": model.register, "mutex": model.mutex}


def _kats():
    cases = json.load(open(GOLDEN))
    for c in cases:
        for op in c["history"]:
            v = op["value"]
            if isinstance(v, dict) and "tuple" in v:
                op["value"] = Tuple(*v["tuple"])
    return cases


@pytest.mark.parametrize("case", _kats(), ids=lambda c: c["name"])
def test_known_answers_on_device(case, tmp_path):
    """etcdemo.clj:115-119 on the device against the hand-derived answers;
    with a store path, linear.svg is drawn for exactly the invalid keys
    (jepsen.checker/linearizable's render-analysis!, lincheck/report.py)."""
    import xml.etree.ElementTree as ET
    mdl = MODELS[case.get("model", "cas-register")]()
    lin = ck.linearizable({"model": mdl, "algorithm": "linear"})
    chk = independent.checker(ck.compose({"linear": lin, "timeline": ck.unbridled_optimism()}))
    out = chk.check({"store-path": str(tmp_path)}, case["history"], {})
    drawn = sorted(int(d) for d in os.listdir(tmp_path / "independent")) if (tmp_path / "independent").exists() else []
    assert drawn == sorted(out["failures"])
    for k in drawn:
        ET.parse(tmp_path / "independent" / str(k) / "linear.svg")
    exp = {int(k): v for k, v in case["expect"].items()}
    assert set(out["results"]) == set(exp)
    bad = sorted(k for k, e in exp.items() if e["valid?"] is False)
    assert sorted(out["failures"]) == bad
    # merge-valid: false > :unknown > true
    unknown = any(e["valid?"] == "unknown" for e in exp.values())
    assert out["valid?"] == (False if bad else "unknown" if unknown else True)
    for k, e in exp.items():
        r = out["results"][k]["linear"]
        assert r["valid?"] == e["valid?"], (case["name"], k)
        if e["valid?"] is False:
            assert r["op"]["index"] == e["op"], (case["name"], k)
            assert r["op"]["type"] == "ok"
            assert r["previous-ok"]["index"] == e["previous-ok"], (case["name"], k)
            assert r["final-paths"], (case["name"], k)


def _wgl_cases():
    """KATs, random multi-key histories (crashes, failures, unmatched
    invocations, nemesis ops), a C5-shaped synthetic one, and VERDICT r3's
    C4-shaped keys: 30 clients, 2 % crashed write/cas, seed 4, 4 keys each at
    300, 600 and 1,200 ops, budget 2^16 -- where :linear gives up on every
    key and WGL's walk decides 7 of 12."""
    out = [(c["name"], c.get("model", "cas-register"), c["history"], 1 << 20) for c in _kats()]
    for seed in range(12):
        out.append((f"random-{seed}", "cas-register",
                    random_history(500 + seed, n_keys=6, max_ops=24, procs=5, p_info=0.05, p_garbage_read=0.15),
                    1 << 20))
    h = H.synth(n_keys=40, ops_per_key=120, concurrency=6, anomaly_rate=0.3, seed=55)
    out.append(("c5-shape", "cas-register", h.to_ops(), 1 << 20))
    for n in (300, 600, 1200):
        h = H.synth(n_keys=4, ops_per_key=n, concurrency=30, info_rate=0.02, seed=4)
        out.append((f"c4-shape-{n}", "cas-register", h.to_ops(), 1 << 16))
    return out


def test_wgl_on_device_against_wgl_restatement():
    """:algorithm :wgl (the slot at etcdemo.clj:118) on the
    device -- knossos.wgl's own walk (device_wgl.hip) -- against
    oracle/wgl_ref.py, the restatement written as knossos.wgl's list walk
    (Wing & Gong with Lowe's cache: a backtracking walk over call / return
    entries).  Per key: :valid? (an :unknown at the cache budget included),
    the :ok the search is stuck on (:op :index), :previous-ok, and :configs
    -- the frontier at that :ok (lc_report_wgl) -- equal to WGL's frontier as
    a set when it has at most 10 configs (jepsen's truncation), a subset of it
    otherwise.  Parity with Knossos itself is unpinned."""
    n_cfg = n_bad = n_c4 = 0
    for name, mname, hist, budget in _wgl_cases():
        mdl = MODELS[mname]()
        lin = ck.linearizable({"model": mdl, "algorithm": "wgl", "max-configs": budget})
        out = independent.checker(lin).check({}, hist, {})
        ref = W.check_independent(hist, budget=budget, model=mname)
        if name.startswith("c4-shape"):
            n_c4 += sum(w.valid is True for w in ref.values())
        assert set(out["results"]) == set(ref), name
        for k, w in ref.items():
            g = out["results"][k]
            if w.cause == "error":
                assert g["valid?"] == "unknown" and "error" in g, (name, k)
                continue
            assert g["valid?"] == w.valid, (name, k)
            assert g["analyzer"] == "wgl", (name, k)
            if w.valid is not False:
                continue
            n_bad += 1
            sub = LR.subhistory(hist, k)
            assert g["op"]["index"] == sub[w.fail_pos]["index"], (name, k)
            prev = g["previous-ok"]["index"] if g["previous-ok"] is not None else None
            assert prev == (sub[w.previous_ok_pos]["index"] if w.previous_ok_pos is not None else None), (name, k)
            idx = lambda oid: sub[w.ops[oid].invoke_pos]["index"]
            want = {(_state_of(mname, st), frozenset(idx(q) for q in lin)) for st, lin in w.frontier}
            got = {(_rendered_state(mname, c["model"]), frozenset(o["index"] for o in c["linearized"]))
                   for c in g["configs"]}
            assert got <= want, (name, k, got - want)
            if len(want) <= 10:
                assert got == want, (name, k)
            n_cfg += len(got)
    assert n_bad > 20 and n_cfg > n_bad
    assert n_c4 >= 7  # decided where :linear gives up


def _state_of(mname, st):
    return bool(st) if mname == "mutex" else st


def _rendered_state(mname, m):
    return m["locked?"] if mname == "mutex" else m["value"]


def test_competition_on_device():
    """The default :algorithm (knossos.competition): the :linear analysis
    answers here (it always finishes), so every KAT and a C5-shaped history
    give exactly the :linear result maps with :analyzer :linear."""
    h = H.synth(n_keys=200, ops_per_key=300, concurrency=10, anomaly_rate=0.1, seed=55)
    histories = [(c["name"], MODELS[c.get("model", "cas-register")](), c["history"]) for c in _kats()]
    histories.append(("c5-shape", model.cas_register(), h.to_ops()))
    for name, mdl, hist in histories:
        ref = independent.checker(ck.linearizable({"model": mdl, "algorithm": "linear"})).check({}, hist, {})
        got = independent.checker(ck.linearizable({"model": mdl})).check({}, hist, {})
        assert _canon(got) == _canon(ref), name


def _canon(out):
    """A result map with :configs and :final-paths as sets (Knossos iterates
    hash sets there; the device's set tiers append in any order)."""
    res = {}
    for k, r in out["results"].items():
        r = dict(r)
        for f in ("configs", "final-paths"):
            if f in r:
                r[f] = sorted(repr(x) for x in r[f])
        res[k] = repr(sorted(r.items()))
    return out["valid?"], sorted(out["failures"]), res


@pytest.mark.parametrize("fmt", ["edn", "fressian"])
@pytest.mark.parametrize("anomaly_rate", [0.0, 0.5])
def test_c1_history_edn_on_device(tmp_path, anomaly_rate, fmt):
    """C1: the demo's shape (6 keys x 100 ops, 10 clients, nemesis :info ops
    every 5 time units, one time-ordered history of tuples) written as
    history.edn, read back by lc_edn_read and checked on the device.  The
    stored run is absent, so the file is synthetic.
    fmt "fressian": the same run as a test.fressian (lc_fressian_write /
    lc_fressian_read) instead."""
    src = H.synth(n_keys=6, ops_per_key=100, concurrency=10, interleave=True, nemesis_period=5.0,
                  anomaly_rate=anomaly_rate, seed=1)
    path = str(tmp_path / ("history.edn" if fmt == "edn" else "test.fressian"))
    write, read = (H.write_edn, H.read_edn) if fmt == "edn" else (H.write_fressian, H.read_fressian)
    write(path, src)
    h = read(path)
    for col in ("type", "f", "process", "key", "v0", "v1", "index"):
        np.testing.assert_array_equal(getattr(h, col), getattr(src, col), err_msg=col)
    assert (h.key == -(1 << 63)).sum() > 0  # the nemesis ops are in the file
    packed = Packed(h)
    res = Device(0).check(packed)
    keys, orc = cref.check_history(h.as_c(), budget=1 << 20, threads=4)
    assert list(keys) == packed.keys
    np.testing.assert_array_equal(res.valid, orc["valid"])
    np.testing.assert_array_equal(res.cause, orc["cause"])
    np.testing.assert_array_equal(res.fail_event, orc["fail_event"])
    # the same file through the demo's checker expression
    lin = ck.linearizable({"model": model.cas_register(), "algorithm": "linear"})
    out = independent.checker(ck.compose({"linear": lin, "timeline": ck.unbridled_optimism()})).check(
        {}, read(path), {})
    fails = sorted(int(k) for k, r in zip(keys, orc) if r["valid"] == 0)
    assert sorted(out["failures"]) == fails
    assert out["valid?"] == (not fails)
    if anomaly_rate:
        assert fails and set(fails) <= set(src.anomalous_keys)


def test_c4_full_size_bench_budget():
    """C4 exactly as bench.py runs it: 256 keys x 5,000 ops, concurrency 30,
    2 % of write/cas crashed (:info), budget 2^16 configs.  Every key's
    :valid?, cause, failing event (and peak set size where the key finished)
    equals the oracle's."""
    budget = 1 << 16
    h = H.synth(n_keys=256, ops_per_key=5000, concurrency=30, info_rate=0.02, seed=4)
    _, res, orc = device_vs_oracle(h, Device(0, budget=budget), budget=budget)
    assert res.stats["deep_keys"] > 0 and res.stats["tier3_ms"] > 0  # the HBM tier ran



@pytest.mark.parametrize("x", [-1, 2**63 - 1])
def test_extreme_register_values_on_device(device, x):
    """a read of -1 on a never-written register is not a
    read of nil; writes of -1 / INT64_MAX are writes of that value.  Device
    verdicts and failing events equal the C restatement's, which reads the
    history itself (tests/test_pack_fast.py has the pack-level check)."""
    from test_pack_fast import _extreme_value_ops
    h = H.History.from_ops(_extreme_value_ops(x))
    _, res, orc = device_vs_oracle(h, device)
    assert list(res.valid) == [0, 1, 0, 1]
