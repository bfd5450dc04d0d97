"""Shared test helpers: run the device and the oracle on the same history."""
import numpy as np

import cref
from lincheck import history as H
from lincheck.checker import Device, Packed

CAUSE = {"none": 0, "nonlin": 1, "budget": 2, "window": 3, "states": 4}


def device_vs_oracle(hist: H.History, dev: Device, budget=None, check_peak=True, verdicts_only=False):
    """Assert bit-exact agreement of the device search with the C restatement.
    verdicts_only: the library's fast path (no sizes, configs or probes asked
    for) -- verdicts, causes and failing events must still be identical."""
    budget = budget or dev.budget
    packed = Packed(hist)
    res = dev.check(packed, verdicts_only=verdicts_only)
    if verdicts_only:
        check_peak = False
    keys, orc = cref.check_history(hist.as_c(), budget=budget, threads=8)
    assert list(keys) == packed.keys
    np.testing.assert_array_equal(res.valid, orc["valid"], err_msg="valid?")
    np.testing.assert_array_equal(res.cause, orc["cause"], err_msg="cause")
    np.testing.assert_array_equal(res.fail_event, orc["fail_event"], err_msg="fail event")
    done = orc["cause"] != CAUSE["budget"]
    if check_peak:
        np.testing.assert_array_equal(res.peak[done], orc["peak"][done], err_msg="peak configs")
    if done.all() and dev.count_probes and not verdicts_only:
        assert res.stats["probes"] == int(orc["probes"].sum())
    return packed, res, orc


# ---- counterexample shaping -----------------------------
def state_ids(packed: Packed, i: int) -> dict:
    """Model-state value -> packed state id for key i (ids may come from a
    table shared by every key, so walk it to its end)."""
    out = {}
    for s in range(1 << 16):
        try:
            out[packed.state_value(i, s)] = s
        except Exception:
            break
    return out


def oracle_state_value(st, model: str):
    """The restatement's state as the value lc_pack interns (mutex: locked -> 1)."""
    if model == "mutex":
        return 1 if st else None
    return st


def encode_finals(packed: Packed, i: int, a, model: str, limit: int = 10):
    """The restatement's final configs in the device's record layout
    (lo = slots 0..63, hi = slots 64..111 | state << 48)."""
    ids = state_ids(packed, i)
    out = np.zeros((limit, 2), np.uint64)
    n = 0
    for st, L in a.final_configs[:limit]:
        mask = 0
        for q in L:
            mask |= 1 << a.final_slots[q]
        out[n, 0] = mask & ((1 << 64) - 1)
        out[n, 1] = (mask >> 64) | (ids[oracle_state_value(st, model)] << 48)
        n += 1
    return out, n


def path_tuple(path, model: str):
    """A rendered :final-paths entry as the restatement's tuple form."""
    def state(m):
        if "msg" in m:
            return "inconsistent"
        v = m["locked?"] if model == "mutex" else m["value"]
        return v
    return tuple(((e["op"]["index"] if e["op"] is not None else None), state(e["model"])) for e in path)


def config_tuple(cfg, model: str):
    """A rendered :configs entry as (state, frozenset of linearized :index)."""
    m = cfg["model"]
    v = m["locked?"] if model == "mutex" else m["value"]
    return (v, frozenset(o["index"] for o in cfg["linearized"]))
