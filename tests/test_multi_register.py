"""(model/multi-register) on the host: the oracle's
restatement against the brute-force definition, and lc_pack's memo (the maps
reachable per key, the transition table) against the restatement's step."""
import numpy as np
import pytest

import brute
import linear_ref as LR
from histgen import multi_register_history, random_history
from lincheck import _native as N
from lincheck import history as H
from lincheck import model
from lincheck.checker import Packed


@pytest.mark.parametrize("seed0", [0, 1000])
def test_oracle_matches_brute_force(seed0):
    """linear_ref's JIT search = the definition, verdict and failing event,
    on random :txn histories (crashes, failures, garbage reads, nemesis)."""
    seen = {True: 0, False: 0}
    for seed in range(seed0, seed0 + 200):
        ops = random_history(seed, n_keys=1, max_ops=7, model="multi-register", p_garbage_read=0.5)
        sub = LR.subhistory(ops, 0)
        a = LR.analysis_safe(sub, model="multi-register")
        v, fe = brute.brute_check(sub, model="multi-register")
        assert (a.valid is True) == v, seed
        assert (a.fail_event if a.valid is False else None) == fe, seed
        seen[v] += 1
    assert seen[True] > 20 and seen[False] > 20


def test_generator_linearizable_by_construction():
    ops = multi_register_history(3, n_keys=30, n_ops=30, corrupt=0.0, p_info=0.05)
    res = LR.check_independent(ops, model="multi-register")
    assert all(r.valid is True for r in res.values())


def _mr_value(st):
    return tuple(sorted(st, key=lambda kv: (str(type(kv[0])), kv[0])))


@pytest.mark.parametrize("init", [None, {"x": 1, "q": 7}])
def test_pack_memo_matches_restatement(init):
    """Per key: key_states = the maps the restatement reaches from the initial
    one under the key's :txn ops, and every table row is the restatement's
    step from every state (LC_TABLE_NONE where inconsistent)."""
    ops = multi_register_history(7, n_keys=12, n_ops=25, corrupt=0.3, p_info=0.05, init=init)
    h = H.History.from_ops(ops)
    mdl = model.multi_register(init)
    pk = Packed(h, mdl)
    v = pk.view
    table = np.ctypeslib.as_array(v.table, shape=(int(v.n_table),))
    trans = np.ctypeslib.as_array(v.trans, shape=(int(v.n_trans),))
    init_t = LR.multi_register_init(init)
    for i, k in enumerate(pk.keys):
        sub = LR.subhistory(ops, k)
        lops, _ = LR.complete(sub, "multi-register")
        S = int(v.key_states[i])
        assert S == LR.reachable_maps(lops, init_t, LR.WIDE_MAX_STATES), k
        states = [_mr_value(pk.state_map(i, s)) for s in range(S)]
        assert states[0] == init_t and len(set(states)) == S
        sid = {st: s for s, st in enumerate(states)}
        # each invoke event's row: the restatement's step of that op
        ev = pk.events(i)
        inv = [j for j in range(len(ev)) if not ev[j] & N.LC_EV_OK_BIT]
        live = [o for o in lops if not o.failed]
        assert len(inv) == len(live)
        for j, o in zip(inv, live):
            row = int(trans[int(v.trans_off[i]) + (int(ev[j]) & 0xFFFFFF)])
            for s, st in enumerate(states):
                nxt = LR.multi_register_step(st, "txn", o.value)
                want = N.LC_TABLE_NONE if nxt is LR.INCONSISTENT else sid[nxt]
                assert int(table[row + s]) == want, (k, j, s)


def test_txn_round_trip_and_errors():
    """:txn values survive History <-> ops; a :txn under (model/cas-register)
    and a micro-op lc_pack cannot step make only their key :unknown (error)."""
    ops = [{"type": "invoke", "f": "txn", "value": H.Tuple(0, [["write", "x", 1]]), "process": 0},
           {"type": "ok", "f": "txn", "value": H.Tuple(0, [["write", "x", 1]]), "process": 0},
           {"type": "invoke", "f": "txn", "value": H.Tuple(1, [["read", 5, None]]), "process": 1},
           {"type": "ok", "f": "txn", "value": H.Tuple(1, [["read", 5, None]]), "process": 1}]
    h = H.History.from_ops(ops)
    back = h.to_ops()
    assert back[0]["value"][1] == [["write", "x", 1]] and back[2]["value"][1] == [["read", 5, None]]
    pk = Packed(h, model.cas_register())
    assert pk.key_error(0) and pk.key_error(1)
    pk = Packed(h, model.multi_register())
    assert pk.key_error(0) is None and int(pk.view.key_states[0]) == 2  # {} and {x 1}
    with pytest.raises(ValueError):
        H.History.from_ops([{"type": "invoke", "f": "txn", "value": [["cas", "x", 1]], "process": 0}])
