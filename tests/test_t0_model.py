"""The register-lattice tier's algorithm, run as a lane-level CPU model
(tests/emu_t0.py: one-directional gathers, lane-masked transfers, Gauss-Seidel
sweeps, lowest-free op indices, two-bit relocation from 7 pending on), must
give the oracle's verdict and failing event on every key it can hold -- both with
exact sets and with the fast path's closed sets (the closure of S under the
pending ops, projected at each :ok).  This
checks the design without a GPU; test_gpu_parity checks the kernel itself."""
import numpy as np
import pytest

import cref
import emu_t0
from lincheck import history as H
from lincheck.checker import Packed


@pytest.mark.parametrize("kw", [
    dict(n_keys=6, ops_per_key=300, concurrency=10, anomaly_rate=0.5, seed=5),
    dict(n_keys=6, ops_per_key=300, concurrency=10, seed=2),
    dict(n_keys=4, ops_per_key=250, concurrency=12, anomaly_rate=0.5, seed=9),
    dict(n_keys=8, ops_per_key=120, concurrency=4, anomaly_rate=0.5, seed=3),
])
@pytest.mark.parametrize("closed", [False, True], ids=["exact", "closed"])
def test_lattice_model_matches_oracle(kw, closed):
    h = H.synth(**kw)
    pk = Packed(h)
    keys, orc = cref.check_history(h.as_c())
    trans = np.ctypeslib.as_array(pk.view.trans, shape=(int(pk.view.n_trans),)).copy()
    held = 0
    for i in range(pk.n_keys):
        r = emu_t0.check_key(pk.events(i), trans, closed=closed)
        if r is None:  # more than 10 pending: the kernel hands such keys to T1
            continue
        held += 1
        assert r == (int(orc["valid"][i]), int(orc["fail_event"][i])), f"key {i}"
    assert held > 0
