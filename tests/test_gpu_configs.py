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
from helpers import device_vs_oracle
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
def test_known_answers_on_device(case):
    """etcdemo.clj:115-119 on the device against the hand-derived answers."""
    mdl = MODELS[case.get("model", "cas-register")]()
    lin = ck.linearizable({"model": mdl, "algorithm": "linear"})
    chk = independent.checker(ck.compose({"linear": lin, "timeline": ck.unbridled_optimism()}))
    out = chk.check({}, case["history"], {})
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


@pytest.mark.parametrize("algo", ["wgl", "competition"])
def test_other_algorithms_on_device(algo):
    """:algorithm :wgl and the default (knossos.competition) on the device
    (SURVEY.md 8(f) F-3): :valid?, the failing-key set and :op :index do not
    depend on the algorithm (the first :ok that cannot be linearized belongs
    to the history), so every KAT and a C5-shaped history give the :linear
    answer; :analyzer names the algorithm that answered."""
    cases = _kats()
    h = H.synth(n_keys=200, ops_per_key=300, concurrency=10, anomaly_rate=0.1, seed=55)
    histories = [(c["name"], MODELS[c.get("model", "cas-register")](), c["history"]) for c in cases]
    histories.append(("c5-shape", model.cas_register(), h.to_ops()))
    for name, mdl, hist in histories:
        outs = {}
        for a in ("linear", algo):
            opts = {"model": mdl} if a == "competition" else {"model": mdl, "algorithm": a}
            outs[a] = independent.checker(ck.linearizable(opts)).check({}, hist, {})
        ref, got = outs["linear"], outs[algo]
        assert got["valid?"] == ref["valid?"], name
        assert sorted(got["failures"]) == sorted(ref["failures"]), name
        for k, r in ref["results"].items():
            g = got["results"][k]
            assert g["valid?"] == r["valid?"], (name, k)
            if "error" not in r:  # check-safe's map for a key that could not be prepared has no analyzer
                assert g["analyzer"] == ("wgl" if algo == "wgl" else "linear"), (name, k)
            if r["valid?"] is False:
                assert g["op"]["index"] == r["op"]["index"], (name, k)
                assert g["previous-ok"]["index"] == r["previous-ok"]["index"], (name, k)


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

