"""The layered HBM tier (device_layers.hip, T3L): entries (L, state mask)
merged one |L| layer at a time in an LDS table, bit-exact with the oracle
(verdict, cause, failing event; peaks and probe counts where keys finish).
Keys with more than 8 register states are handed to the config-keyed narrow
tier, keys needing window slots >= 56 to the wide one; LC_PATH_LAYERS_OFF (the
config-keyed narrow tier alone) must give the same records."""
import numpy as np
import pytest

from helpers import device_vs_oracle
from lincheck import _native as N
from lincheck import history as H
from lincheck.checker import Device, Packed

pytestmark = pytest.mark.gpu


def _same_records(h, budget, count_probes=False):
    """The layered and the config-keyed narrow tiers on one history."""
    p = Packed(h)
    a = Device(0, budget=budget, count_probes=count_probes).check(p)
    b = Device(0, budget=budget, count_probes=count_probes, path_flags=N.LC_PATH_LAYERS_OFF).check(p)
    for f in ("valid", "cause", "fail_event"):
        np.testing.assert_array_equal(getattr(a, f), getattr(b, f), err_msg=f)
    return a, b


@pytest.mark.parametrize("budget", [1 << 12, 1 << 16])
def test_c4_shape_layers(budget):
    """C4's shape (concurrency 30, 2 % crashed write/cas): frontier blow-up
    in the layered tier, :unknown at the oracle's event."""
    h = H.synth(n_keys=32, ops_per_key=1500, concurrency=30, info_rate=0.02, seed=41)
    _, res, orc = device_vs_oracle(h, Device(0, budget=budget, count_probes=True), budget=budget)
    assert res.stats["deep_keys"] > 0 and res.stats["tier3_ms"] > 0
    assert (orc["cause"] == 2).any()


@pytest.mark.parametrize("conc,info,seed", [(20, 0.005, 31), (16, 0.01, 32), (18, 0.01, 33)])
def test_layers_finish_with_peaks_and_probes(conc, info, seed):
    """Keys that finish (valid / invalid, 10^3-10^5 configs) in the layered
    tier: peaks and the total probe count equal the oracle's too."""
    h = H.synth(n_keys=32, ops_per_key=600, concurrency=conc, info_rate=info, anomaly_rate=0.1, seed=seed)
    dev = Device(0, budget=1 << 20, count_probes=True)
    _, res, orc = device_vs_oracle(h, dev, budget=1 << 20)
    assert res.stats["deep_keys"] > 0
    assert (orc["cause"] != 2).all() and orc["peak"].max() > 2048


def test_layers_large_layers_multi_pass():
    """A 2^20 budget on C4-shaped keys: layers far larger than the LDS table
    (multi-pass merges, redone passes) before the budget ends the key."""
    budget = 1 << 20
    h = H.synth(n_keys=6, ops_per_key=1500, concurrency=30, info_rate=0.02, seed=42)
    _, res, orc = device_vs_oracle(h, Device(0, budget=budget), budget=budget)
    assert res.stats["deep_keys"] > 0


def test_layers_hand_on_many_states():
    """12 register values (13 states > 8): the layered tier hands the keys to
    the config-keyed narrow tier; still bit-exact."""
    h = H.synth(n_keys=24, ops_per_key=600, concurrency=18, info_rate=0.01, n_values=12, seed=43)
    _, res, _ = device_vs_oracle(h, Device(0, budget=1 << 18, count_probes=True), budget=1 << 18)
    assert res.stats["deep_keys"] > 0


def test_layers_match_config_keyed_tier():
    h = H.synth(n_keys=48, ops_per_key=1200, concurrency=24, info_rate=0.015, anomaly_rate=0.1, seed=44)
    a, b = _same_records(h, 1 << 16)
    assert a.stats["deep_keys"] > 0


def test_layers_final_configs(device):
    """Invalid keys decided in the layered tier return final configs drawn from
    the set standing before the failing :ok (checked by the oracle's
    enumeration in test_counterexamples for the other tiers; here: same
    records as the config-keyed tier's set, as sets)."""
    h = H.synth(n_keys=40, ops_per_key=400, concurrency=16, info_rate=0.01, anomaly_rate=0.5, seed=45)
    p = Packed(h)
    a = Device(0, budget=1 << 20).check(p)
    b = Device(0, budget=1 << 20, path_flags=N.LC_PATH_LAYERS_OFF).check(p)
    bad = np.nonzero(a.valid == 0)[0]
    assert len(bad) > 0
    np.testing.assert_array_equal(a.fail_event, b.fail_event)
    for i in bad:
        na, nb = int(a.n_final[i]), int(b.n_final[i])
        assert na == nb
        fa = {tuple(r) for r in a.final[i][:na].tolist()}
        fb = {tuple(r) for r in b.final[i][:nb].tolist()}
        if na < 10:  # the whole set: equal
            assert fa == fb
