"""Key segments (device_lattice.hip, "Key segments"): verdict-only
register-tier steps over about one key per SIMD cut each key at quiescent
points, search every segment from all start states at once (tagged lattice
words) and compose per key; a key that dies is searched again, untagged, in
the segment it died in.  Verdicts, causes and failing events must equal the
oracle's and the unsplit search's, whatever the segment length."""
import numpy as np
import pytest

import cref
from lincheck import _native as N
from lincheck import history as H
from lincheck.checker import Device, Packed

pytestmark = pytest.mark.gpu

SHAPES = {
    "c2": dict(n_keys=400, ops_per_key=1000, concurrency=10, seed=81),
    "c5": dict(n_keys=400, ops_per_key=1000, concurrency=10, anomaly_rate=0.2, seed=82),
    "late_anomalies": dict(n_keys=200, ops_per_key=2000, concurrency=8, anomaly_rate=0.5, seed=83),
    "low_concurrency": dict(n_keys=300, ops_per_key=800, concurrency=3, anomaly_rate=0.2, seed=84),
    "crashed": dict(n_keys=300, ops_per_key=800, concurrency=6, info_rate=0.002, anomaly_rate=0.2, seed=85),
    "two_values": dict(n_keys=300, ops_per_key=800, concurrency=9, n_values=2, anomaly_rate=0.2, seed=86),
}


@pytest.mark.parametrize("shape", sorted(SHAPES))
@pytest.mark.parametrize("seg_len", [0, 64, 1])
def test_segments_match_oracle(shape, seg_len):
    h = H.synth(**SHAPES[shape])
    pk = Packed(h)
    got = Device(0, path_flags=N.LC_PATH_SPLIT_ON, seg_len=seg_len).check(pk, verdicts_only=True)
    ref = Device(0, path_flags=N.LC_PATH_SPLIT_OFF).check(pk, verdicts_only=True)
    _, orc = cref.check_history(h.as_c(), budget=1 << 20, threads=8)
    for name, r in (("split", got), ("unsplit", ref)):
        np.testing.assert_array_equal(r.valid, orc["valid"], err_msg=f"{name} valid")
        np.testing.assert_array_equal(r.cause, orc["cause"], err_msg=f"{name} cause")
        np.testing.assert_array_equal(r.fail_event, orc["fail_event"], err_msg=f"{name} fail_event")
    if SHAPES[shape].get("anomaly_rate"):
        assert (orc["valid"] == 0).any()


def test_segments_resident_async():
    """The bench's resident steps (node records, asynchronous) on the split path."""
    h = H.synth(n_keys=1000, ops_per_key=1000, concurrency=10, anomaly_rate=0.05, seed=87)
    pk = Packed(h)
    dev = Device(0, path_flags=N.LC_PATH_SPLIT_ON)
    db = dev.upload(pk)
    for _ in range(5):
        db.check_node(pk.n_keys, asynchronous=True)
    dev.wait()
    rec = dev.node_records(pk.n_keys).astype(np.int64)
    _, orc = cref.check_history(h.as_c(), budget=dev.budget, threads=8)
    np.testing.assert_array_equal((rec & 0xFF) - 1, orc["valid"])
    np.testing.assert_array_equal((rec >> 16) - 1, orc["fail_event"])


def test_low_overlap_split_by_default():
    """Clients that think longer than an op takes (the demo's 10 Hz per
    thread against millisecond latencies): quiescent points are frequent,
    the default choice cuts the keys, and the verdicts equal the oracle's."""
    h = H.synth(n_keys=64, ops_per_key=4000, concurrency=10, mean_think=20.0, anomaly_rate=0.25, seed=88)
    pk = Packed(h)
    dev = Device(0)
    got = dev.check(pk, verdicts_only=True)
    _, orc = cref.check_history(h.as_c(), budget=dev.budget, threads=8)
    np.testing.assert_array_equal(got.valid, orc["valid"])
    np.testing.assert_array_equal(got.fail_event, orc["fail_event"])
    assert (orc["valid"] == 0).any()
