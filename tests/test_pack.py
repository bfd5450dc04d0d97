"""lc_pack (jepsen.independent split + knossos.history complete /
without-failures + memoised cas-register transitions) against the oracle's
own restatement of the same steps (oracle/linear_ref.py)."""
import ctypes as C

import numpy as np
import pytest
from hypothesis import given, settings, strategies as st

import linear_ref as LR
from histgen import random_history
from lincheck import _native as N
from lincheck import history as H
from lincheck.checker import Packed
from lincheck.independent import Tuple


def decode(desc):
    return desc & 3, (desc >> 2) & 0x7FFF, desc >> 17


def check_packed_against_oracle(ops):
    h = H.History.from_ops(ops)
    pk = Packed(h)
    assert pk.keys == LR.history_keys(ops)
    view = pk.view
    trans = np.ctypeslib.as_array(view.trans, shape=(view.n_trans,))
    toff = None if not view.trans_off else np.ctypeslib.as_array(view.trans_off, shape=(pk.n_keys,))
    width = np.ctypeslib.as_array(view.key_width, shape=(pk.n_keys,))
    for i, k in enumerate(pk.keys):
        sub = LR.subhistory(ops, k)
        lops, events = LR.complete(sub)
        # sub-history rows: tuple rows of k + shared (nemesis) rows, in order
        nrows = N.lib().lc_packed_subhistory(pk.handle, i, None)
        rows = np.zeros(max(nrows, 1), np.int64)
        N.lib().lc_packed_subhistory(pk.handle, i, N.ptr(rows, C.c_int64))
        rows = rows[:nrows]
        assert len(rows) == len(sub)
        ev = pk.events(i)
        assert len(ev) == len(events)
        free = list(range(128))
        slot_of = {}
        maxw = 0
        for j, (kind, oid, pos) in enumerate(events):
            w = int(ev[j])
            assert pk.event_row(i, j) == rows[pos]
            if kind == "invoke":
                assert not w & N.LC_EV_OK_BIT
                s = min(free); free.remove(s); slot_of[oid] = s
                maxw = max(maxw, s + 1)
                assert (w >> 24) & 0x7F == s
                f, a, b = decode(int(trans[(0 if toff is None else toff[i]) + (w & 0xFFFFFF)]))
                o = lops[oid]
                val = lambda sid: pk.state_value(i, sid) if sid != N.LC_STATE_NONE else "NONE"
                if o.f == "read":
                    if o.value is None:
                        assert f == N.LC_T_READ_ANY
                    else:
                        assert f == N.LC_T_READ and val(a) in (o.value, "NONE")
                elif o.f == "write":
                    assert f == N.LC_T_WRITE and val(b) == o.value
                else:
                    assert f == N.LC_T_CAS and val(b) == o.value[1] and val(a) in (o.value[0], "NONE")
            else:
                assert w & N.LC_EV_OK_BIT
                s = slot_of.pop(oid)
                assert (w >> 24) & 0x7F == s
                free.append(s)
        assert width[i] == maxw


@settings(max_examples=150, deadline=None)
@given(st.integers(0, 2**31 - 1))
def test_pack_matches_restatement_random(seed):
    check_packed_against_oracle(random_history(seed, n_keys=3, max_ops=10, procs=4))


@pytest.mark.parametrize("kw", [
    dict(n_keys=5, ops_per_key=100, concurrency=10, seed=2),
    dict(n_keys=3, ops_per_key=100, concurrency=30, info_rate=0.05, seed=4),
    dict(n_keys=4, ops_per_key=80, concurrency=10, interleave=True, nemesis_period=2.0, seed=1),
    dict(n_keys=3, ops_per_key=200, concurrency=4, n_values=400, seed=8),   # per-key state tables
])
def test_pack_matches_restatement_synthetic(kw):
    check_packed_against_oracle(H.synth(**kw).to_ops())


def test_many_values_use_per_key_tables():
    h = H.synth(n_keys=3, ops_per_key=400, concurrency=4, n_values=1000, seed=8)
    pk = Packed(h)
    assert pk.view.trans_off  # > 254 distinct values: per-key state numbering
    states = np.ctypeslib.as_array(pk.view.key_states, shape=(pk.n_keys,))
    assert (states > 100).all()


def test_completion_without_invocation_is_a_key_error():
    """complete's assertion fails for key 1 only: that key keeps its place with
    no events and an error (check-safe per key, etcdemo.clj:115); key 0 packs
    as usual."""
    ops = [{"type": "invoke", "f": "write", "value": Tuple(0, 1), "process": 0},
           {"type": "ok", "f": "write", "value": Tuple(1, 1), "process": 1},
           {"type": "ok", "f": "write", "value": Tuple(0, 1), "process": 0}]
    pk = Packed(H.History.from_ops(ops))
    assert pk.keys == [0, 1]
    assert pk.key_error(0) is None
    assert "without a prior invocation" in pk.key_error(1)
    assert pk.n_events(0) == 2 and pk.n_events(1) == 0
    err = np.ctypeslib.as_array(pk.view.key_error, shape=(2,))
    assert list(err) == [0, 1]


def test_no_key_errors_no_array():
    pk = Packed(H.synth(n_keys=3, ops_per_key=20, concurrency=3, seed=1))
    assert not pk.view.key_error


def test_non_tuple_client_op_in_every_key():
    """jepsen.independent/subhistory keeps non-tuple ops: an un-keyed write is
    an op of every key's sub-history."""
    ops = [{"type": "invoke", "f": "write", "value": Tuple(0, 1), "process": 0},
           {"type": "ok", "f": "write", "value": Tuple(0, 1), "process": 0},
           {"type": "invoke", "f": "write", "value": 3, "process": 9},
           {"type": "ok", "f": "write", "value": 3, "process": 9},
           {"type": "invoke", "f": "read", "value": Tuple(1, None), "process": 1},
           {"type": "ok", "f": "read", "value": Tuple(1, 3), "process": 1}]
    pk = Packed(H.History.from_ops(ops))
    assert pk.keys == [0, 1]
    assert [pk.n_events(i) for i in range(2)] == [4, 4]
    assert [pk.event_row(1, j) for j in range(4)] == [2, 3, 4, 5]
    check_packed_against_oracle(ops)


def test_unknown_f_is_a_key_error():
    ops = [{"type": "invoke", "f": "append", "value": Tuple(0, 1), "process": 0},
           {"type": "invoke", "f": "write", "value": Tuple(1, 1), "process": 1}]
    pk = Packed(H.History.from_ops(ops))
    assert "cannot step" in pk.key_error(0) and pk.key_error(1) is None


def test_non_integer_values_rejected_on_host():
    with pytest.raises(ValueError):
        H.History.from_ops([{"type": "invoke", "f": "write", "value": Tuple(0, "x"), "process": 0}])


def test_empty_history():
    pk = Packed(H.History.from_ops([]))
    assert pk.n_keys == 0


def test_double_invoke_leaves_first_pending_forever():
    ops = [{"type": "invoke", "f": "write", "value": Tuple(0, 1), "process": 0},
           {"type": "invoke", "f": "write", "value": Tuple(0, 2), "process": 0},
           {"type": "ok", "f": "write", "value": Tuple(0, 2), "process": 0}]
    pk = Packed(H.History.from_ops(ops))
    ev = pk.events(0)
    assert [(int(w) >> 31, (int(w) >> 24) & 0x7F) for w in ev] == [(0, 0), (0, 1), (1, 1)]


def test_models_pack():
    """(model/mutex) packs acquire / release as cas over {unlocked, locked};
    (model/register) refuses a cas, as knossos's Register cannot step it."""
    from lincheck import _native as N
    from lincheck import model
    from lincheck.checker import Packed
    from lincheck.independent import Tuple
    ops = [{"type": "invoke", "f": "acquire", "value": Tuple(0, None), "process": 0},
           {"type": "ok", "f": "acquire", "value": Tuple(0, None), "process": 0},
           {"type": "invoke", "f": "release", "value": Tuple(0, None), "process": 0},
           {"type": "ok", "f": "release", "value": Tuple(0, None), "process": 0}]
    pk = Packed(H.History.from_ops(ops), model.mutex())
    trans = np.ctypeslib.as_array(pk.view.trans, shape=(int(pk.view.n_trans),))
    assert sorted(int(t) for t in trans) == sorted([N.LC_T_CAS | (0 << 2) | (1 << 17), N.LC_T_CAS | (1 << 2) | (0 << 17)])
    cas = [{"type": "invoke", "f": "cas", "value": Tuple(0, [1, 2]), "process": 0}]
    assert "cannot step" in Packed(H.History.from_ops(cas), model.register()).key_error(0)
    assert "cannot step" in Packed(H.History.from_ops(ops), model.cas_register()).key_error(0)


def test_events16_widen_to_events():
    """lc_pack's 16-bit event words (lc_batch.events16) widen to exactly the
    32-bit words (LC_EV16_WIDE), and are omitted when a word does not fit."""
    import numpy as np
    from lincheck.checker import Packed
    pk = Packed(H.synth(n_keys=50, ops_per_key=200, concurrency=10, anomaly_rate=0.2, seed=9))
    n = int(pk.ev_off[-1])
    # the 16-bit words are the batch's (ABI 11: no 32-bit copy beside them;
    # tests/test_pack_fast.py holds them to the bucketing path's)
    assert not pk.view.events
    e16 = np.ctypeslib.as_array(pk.view.events16, shape=(n,)).astype(np.uint32)
    wide = ((e16 & 0x8000) << 16) | (((e16 >> 11) & 0xF) << 24) | (e16 & 0x7FF)
    np.testing.assert_array_equal(pk.all_events(), wide)
    # > 16 ops pending at once: slots past 15, no 16-bit form
    pk = Packed(H.synth(n_keys=4, ops_per_key=300, concurrency=40, mean_think=0.1, seed=9))
    assert not pk.view.events16
