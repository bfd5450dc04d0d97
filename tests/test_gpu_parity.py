"""Device search vs the C restatement of knossos.linear -- bit-exact parity.

Every case runs the same seeded history through liblincheck.so (the HIP
path) and oracle/linear_ref.c and compares, per key: :valid?, the cause, the
failing event, the peak config-set size, and the total probe count.
"""
import numpy as np
import pytest

from helpers import device_vs_oracle
from lincheck import history as H
from lincheck.checker import Device

pytestmark = pytest.mark.gpu


def test_c2_shape_all_valid(device):
    h = H.synth(n_keys=300, ops_per_key=1000, concurrency=10, seed=2)
    _, res, _ = device_vs_oracle(h, device)
    assert (res.valid == 1).all()


def test_c5_shape_anomalies(device):
    h = H.synth(n_keys=400, ops_per_key=1000, concurrency=10, anomaly_rate=0.05, seed=5)
    _, res, _ = device_vs_oracle(h, device)
    assert (res.valid == 0).sum() > 0


def test_small_keys_many(device):
    h = H.synth(n_keys=3000, ops_per_key=40, concurrency=5, anomaly_rate=0.2, seed=11)
    device_vs_oracle(h, device)


def test_tight_budget_unknown(device):
    dev = Device(0, budget=48)
    h = H.synth(n_keys=200, ops_per_key=500, concurrency=10, anomaly_rate=0.1, seed=13)
    _, res, _ = device_vs_oracle(h, dev, budget=48)
    assert (res.valid == -1).sum() > 0


def test_high_concurrency_spills_to_t2(device):
    h = H.synth(n_keys=64, ops_per_key=600, concurrency=16, seed=17)
    _, res, _ = device_vs_oracle(h, device)
