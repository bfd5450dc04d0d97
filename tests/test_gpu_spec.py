"""Speculative key segments (device_lattice.hip, "Speculative key segments"):
verdict-only register-tier steps of about one key per SIMD or fewer search
every key as a workgroup of segment waves -- each segment from the full
config set, then again from its predecessor's end set until the two runs
meet -- and walk the segments in order.  Verdicts, causes and failing events
must equal the oracle's and the unsegmented search's, whatever the segment
count and checkpoint distances (tiny distances make runs miss each other and
exercise the fallback to the unsegmented search)."""
import numpy as np
import pytest

import cref
from lincheck import _native as N
from lincheck import history as H
from lincheck.checker import Device, Packed

pytestmark = pytest.mark.gpu

SHAPES = {
    "c2": dict(n_keys=400, ops_per_key=1000, concurrency=10, seed=91),
    "c5": dict(n_keys=400, ops_per_key=1000, concurrency=10, anomaly_rate=0.2, seed=92),
    "late_anomalies": dict(n_keys=200, ops_per_key=2000, concurrency=8, anomaly_rate=0.5, seed=93),
    "low_concurrency": dict(n_keys=300, ops_per_key=800, concurrency=3, anomaly_rate=0.2, seed=94),
    "crashed": dict(n_keys=300, ops_per_key=800, concurrency=6, info_rate=0.002, anomaly_rate=0.2, seed=95),
    "two_values": dict(n_keys=300, ops_per_key=800, concurrency=9, n_values=2, anomaly_rate=0.2, seed=96),
    "wide": dict(n_keys=200, ops_per_key=1500, concurrency=10, mean_think=0.3, anomaly_rate=0.2, seed=97),
    "short_keys": dict(n_keys=500, ops_per_key=150, concurrency=10, anomaly_rate=0.2, seed=98),
    "think20": dict(n_keys=64, ops_per_key=3000, concurrency=10, mean_think=20.0, anomaly_rate=0.25, seed=99),
}


def _check(dev, pk, orc, what):
    r = dev.check(pk, verdicts_only=True)
    np.testing.assert_array_equal(r.valid, orc["valid"], err_msg=f"{what}: valid")
    np.testing.assert_array_equal(r.cause, orc["cause"], err_msg=f"{what}: cause")
    np.testing.assert_array_equal(r.fail_event, orc["fail_event"], err_msg=f"{what}: fail_event")


@pytest.mark.parametrize("shape", sorted(SHAPES))
def test_spec_matches_oracle(shape):
    h = H.synth(**SHAPES[shape])
    pk = Packed(h)
    _, orc = cref.check_history(h.as_c(), budget=1 << 20, threads=8)
    _check(Device(0, path_flags=N.LC_PATH_SPLIT_OFF | N.LC_PATH_SPEC_OFF), pk, orc, "unsegmented")
    for segs in (2, 3, 4, 6, 8):
        for ck in ((32, 160), (1, 2), (0, 0)):
            dev = Device(0, path_flags=N.LC_PATH_SPLIT_OFF, spec_segs=segs, spec_ck=ck)
            _check(dev, pk, orc, f"segs {segs} ck {ck}")
    # the other cut placement (equal estimated cost), the 32-bit words, age priority
    for flags in (N.LC_PATH_SPEC_COST, N.LC_PATH_EV32, N.LC_PATH_SPEC_NOPRIO):
        dev = Device(0, path_flags=N.LC_PATH_SPLIT_OFF | flags, spec_segs=4)
        _check(dev, pk, orc, f"segs 4, path_flags {flags:#x}")
    if SHAPES[shape].get("anomaly_rate"):
        assert (orc["valid"] == 0).any()


def test_spec_reruns_walk_the_rerun_grid():
    """More keys left to the unsegmented search than the rerun launch has
    waves (k_spec_rerun runs one 4-wave workgroup per CU, 1,024 waves on the
    MI355X): checkpoints at the cut make runs miss each other, so most of the
    3,000 keys go through the rerun kernel's grid-stride loop -- verdicts,
    causes and failing events still the oracle's."""
    h = H.synth(n_keys=3000, ops_per_key=300, concurrency=10, anomaly_rate=0.2, seed=102)
    pk = Packed(h)
    _, orc = cref.check_history(h.as_c(), budget=1 << 20, threads=8)
    for segs in (2, 4):
        dev = Device(0, path_flags=N.LC_PATH_SPLIT_OFF, spec_segs=segs, spec_ck=(0, 0))
        _check(dev, pk, orc, f"reruns, segs {segs}")
    assert (orc["valid"] == 0).any()


def test_spec_default_on_c2_shape():
    """The default choice for a C2-sized verdicts-only batch is the
    speculative path (checked through its result only: same as the oracle)."""
    h = H.synth(n_keys=1000, ops_per_key=1000, concurrency=10, anomaly_rate=0.05, seed=100)
    pk = Packed(h)
    dev = Device(0)
    _, orc = cref.check_history(h.as_c(), budget=dev.budget, threads=8)
    _check(dev, pk, orc, "default")


def test_spec_resident_async():
    """The bench's resident steps (node records, asynchronous) on the speculative path."""
    h = H.synth(n_keys=1000, ops_per_key=1000, concurrency=10, anomaly_rate=0.05, seed=101)
    pk = Packed(h)
    dev = Device(0)
    db = dev.upload(pk)
    for _ in range(5):
        db.check_node(pk.n_keys, asynchronous=True)
    dev.wait()
    rec = dev.node_records(pk.n_keys).astype(np.int64)
    _, orc = cref.check_history(h.as_c(), budget=dev.budget, threads=8)
    np.testing.assert_array_equal((rec & 0xFF) - 1, orc["valid"])
    np.testing.assert_array_equal((rec >> 16) - 1, orc["fail_event"])


def _finals(r, k):
    n = min(int(r.n_final[k]), r.final.shape[1])
    return sorted(map(tuple, r.final[k, :n].tolist()))


@pytest.mark.parametrize("shape", ["c5", "crashed", "two_values", "think20", "short_keys"])
def test_exact_spec_final_configs(shape):
    """Final configs without peak sizes (the Knossos-shaped checkers) run the
    segments with exact sets (k_spec<.., EX>): verdicts, causes, failing
    events, final-config counts and the final config records equal the
    unsegmented exact search's, whatever the segment count and checkpoints
    (records are the smallest in (slot mask, state) order, so a run's own
    op-index assignment does not change which ones are kept)."""
    h = H.synth(**SHAPES[shape])
    pk = Packed(h)
    _, orc = cref.check_history(h.as_c(), budget=1 << 20, threads=8)
    for mf in (10, 16):
        ref = Device(0, path_flags=N.LC_PATH_SPLIT_OFF | N.LC_PATH_SPEC_OFF, max_final=mf).check(pk, peaks=False)
        np.testing.assert_array_equal(ref.valid, orc["valid"])
        np.testing.assert_array_equal(ref.fail_event, orc["fail_event"])
        runs = [("default", dict())]
        runs += [(f"segs {s} ck {ck}", dict(path_flags=N.LC_PATH_SPLIT_OFF, spec_segs=s, spec_ck=ck))
                 for s in (2, 4, 8) for ck in ((32, 120), (1, 2))] if mf == 10 else []
        for what, kw in runs:
            r = Device(0, max_final=mf, **kw).check(pk, peaks=False)
            assert r.stats["t0_path"] == "k_spec", what
            for f in ("valid", "cause", "fail_event", "n_final"):
                np.testing.assert_array_equal(getattr(r, f), getattr(ref, f), err_msg=f"{what}, max_final {mf}: {f}")
            # the records written, in order (the rest of each row is not written)
            bad = [k for k in range(pk.n_keys) if r.final[k, :r.n_final[k]].tolist() != ref.final[k, :ref.n_final[k]].tolist()]
            assert not bad, f"{what}, max_final {mf}: final configs differ on keys {bad[:8]}"
    if SHAPES[shape].get("anomaly_rate"):
        assert (ref.valid == 0).any()
