"""Shared test helpers: run the device and the oracle on the same history."""
import numpy as np

import cref
from lincheck import history as H
from lincheck.checker import Device, Packed

CAUSE = {"none": 0, "nonlin": 1, "budget": 2, "window": 3, "states": 4}


def device_vs_oracle(hist: H.History, dev: Device, budget=None, check_peak=True):
    """Assert bit-exact agreement of the device search with the C restatement."""
    budget = budget or dev.budget
    packed = Packed(hist)
    res = dev.check(packed)
    keys, orc = cref.check_history(hist.as_c(), budget=budget, threads=8)
    assert list(keys) == packed.keys
    np.testing.assert_array_equal(res.valid, orc["valid"], err_msg="valid?")
    np.testing.assert_array_equal(res.cause, orc["cause"], err_msg="cause")
    np.testing.assert_array_equal(res.fail_event, orc["fail_event"], err_msg="fail event")
    done = orc["cause"] != CAUSE["budget"]
    if check_peak:
        np.testing.assert_array_equal(res.peak[done], orc["peak"][done], err_msg="peak configs")
    if done.all() and dev.count_probes:
        assert res.stats["probes"] == int(orc["probes"].sum())
    return packed, res, orc
