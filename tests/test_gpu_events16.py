"""16-bit event words on the device (lc_batch.events16): a register-tier
batch uploaded at 2 bytes per event and widened on the GPU gives the same
records as the 32-bit upload, in every path that takes it (lc_check_node,
lc_check_batch, lc_upload + resident steps), and the oracle's verdicts."""
import ctypes as C

import numpy as np
import pytest

import cref
from lincheck import _native as N
from lincheck import history as H
from lincheck import parallel as P
from lincheck.checker import Device, Packed

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("keys,ops,anom", [(300, 1000, 0.05), (5000, 120, 0.1)])
def test_events16_same_records(keys, ops, anom):
    h = H.synth(n_keys=keys, ops_per_key=ops, concurrency=10, anomaly_rate=anom, seed=41)
    pk = Packed(h)
    assert pk.view.events16  # the batch fits 16 bits
    dev = Device(0)
    rec16, _ = dev.check_node(pk, keys)
    rec16 = rec16.copy()
    r16 = dev.check(pk, verdicts_only=True)
    db = dev.upload(pk)
    db.check_node(keys, asynchronous=True)
    dev.wait()
    res16 = dev.node_records(keys)
    del db
    # the 32-bit upload: the same words widened on the host (lc_pack gives
    # only the 16-bit ones when every word fits, ABI 11)
    e32 = pk.all_events()
    saved = (pk.view.events, pk.view.events16)
    pk.view.events, pk.view.events16 = N.ptr(e32, C.c_uint32), None
    rec32, _ = dev.check_node(pk, keys)
    r32 = dev.check(pk, verdicts_only=True)
    pk.view.events, pk.view.events16 = saved
    np.testing.assert_array_equal(rec16, rec32)
    np.testing.assert_array_equal(res16, rec32)
    np.testing.assert_array_equal(r16.valid, r32.valid)
    np.testing.assert_array_equal(r16.fail_event, r32.fail_event)
    _, orc = cref.check_history(h.as_c(), threads=8)
    v, c, fe = P.unpack_records(rec16.astype(np.int64))
    np.testing.assert_array_equal(v, orc["valid"])
    np.testing.assert_array_equal(fe, orc["fail_event"])
