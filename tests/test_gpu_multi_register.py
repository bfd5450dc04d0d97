"""(model/multi-register) on the device: lc_pack's
transition table through the set tiers (T1/T2 in LDS, T3 in HBM, wide
configs past 255 maps), against the restatement (oracle/linear_ref.py) on the
same histories -- verdicts, failing events, peak set sizes, and the rendered
:op / :previous-ok / :final-paths of independent/checker."""
import numpy as np
import pytest

import linear_ref as LR
from histgen import multi_register_history
from lincheck import checker as ck
from lincheck import history as H
from lincheck import independent, model
from lincheck.checker import Device, Packed

pytestmark = pytest.mark.gpu

SHAPES = {
    # registers x values -> maps per key; procs -> ops pending at once
    "narrow": dict(seed=11, n_keys=40, n_ops=50, procs=5, regs=("x", "y", "z"), values=(0, 1, 2, 3)),
    "crashed": dict(seed=12, n_keys=24, n_ops=40, procs=6, regs=("x", "y"), values=(0, 1, 2), p_info=0.12),
    "wide_states": dict(seed=13, n_keys=12, n_ops=60, procs=4, regs=(1, 2, 3, 4), values=(0, 1, 2, 3, 4)),
    "init_map": dict(seed=14, n_keys=30, n_ops=40, procs=5, regs=("x", "y"), values=(0, 1, 2), init={"x": 0, "w": 9}),
}


def _path(p):
    out = []
    for e in p:
        m = e["model"]
        st = "inconsistent" if "msg" in m else tuple(sorted(m.items(), key=lambda kv: (str(type(kv[0])), kv[0])))
        out.append(((e["op"]["index"] if e["op"] is not None else None), st))
    return tuple(out)


@pytest.mark.parametrize("budget", [1 << 20, 24])
@pytest.mark.parametrize("shape", sorted(SHAPES))
def test_multi_register_on_device(shape, budget):
    kw = dict(SHAPES[shape])
    init = kw.pop("init", None)
    ops = multi_register_history(corrupt=0.3, init=init, **kw)
    mdl = model.multi_register(init)
    orc = LR.check_independent(ops, budget=budget, model="multi-register", initial=LR.multi_register_init(init))
    # the device's records against the restatement's, key by key
    pk = Packed(H.History.from_ops(ops), mdl)
    res = Device(0, budget=budget).check(pk)
    want_v = {True: 1, False: 0, "unknown": -1}
    for i, k in enumerate(pk.keys):
        a = orc[k]
        assert int(res.valid[i]) == want_v[a.valid], (shape, k, a.cause)
        assert int(res.fail_event[i]) == (a.fail_event if a.fail_event is not None else -1), (shape, k)
        if a.cause != "budget":
            assert int(res.peak[i]) == a.peak_configs, (shape, k)
    if shape == "wide_states":
        assert int(pk.view.key_states[0]) > 255  # wide configs (the HBM tier)
    if budget == 1 << 20:
        assert (res.valid == 0).any() and (res.valid == 1).any()
    else:
        assert (res.valid == -1).any()  # the budget ends keys (identically)
    # the checker expression of etcdemo.clj:115-119 with the other model
    lin = ck.linearizable({"model": mdl, "algorithm": "linear", "max-configs": budget})
    out = independent.checker(lin).check({}, ops, {})
    bad = sorted(k for k, a in orc.items() if a.valid is False)
    assert sorted(out["failures"]) == bad
    for k in bad:
        a, r = orc[k], out["results"][k]
        sub = LR.subhistory(ops, k)
        assert r["op"]["index"] == sub[a.fail_pos]["index"]
        prev = sub[a.previous_ok_pos]["index"] if a.previous_ok_pos is not None else None
        assert (r["previous-ok"] or {}).get("index") == prev
        paths = {_path(p) for p in r["final-paths"]}
        allp = LR.final_paths(a, sub, model="multi-register")
        if allp is not None:
            assert paths <= allp
            if len(allp) <= ck.TRUNCATE:
                assert paths == allp


def test_multi_register_history_edn_on_device(tmp_path):
    """The same kind of history as a history.edn file (keyword registers,
    [k txn] tuples), read by lc_edn_read and checked on the device: verdicts
    and failing events equal the restatement's on the op maps."""
    from test_edn import _txn_lines
    ops = multi_register_history(21, n_keys=30, n_ops=40, procs=5, regs=("x", "y", "z"), values=(0, 1, 2, 3),
                                 corrupt=0.3, p_info=0.05)
    for i, o in enumerate(ops):
        o["index"] = i
    path = tmp_path / "history.edn"
    path.write_text(_txn_lines(ops))
    h = H.read_edn(str(path))
    pk = Packed(h, model.multi_register())
    res = Device(0).check(pk)
    orc = LR.check_independent(ops, model="multi-register")
    want_v = {True: 1, False: 0, "unknown": -1}
    for i, k in enumerate(pk.keys):
        assert int(res.valid[i]) == want_v[orc[k].valid], k
        assert int(res.fail_event[i]) == (orc[k].fail_event if orc[k].fail_event is not None else -1), k
    assert (res.valid == 0).any() and (res.valid == 1).any()
