"""Diagnose exact speculative segments vs the unsegmented exact search on one shape."""
import sys
import numpy as np
sys.path.insert(0, "tests")
sys.path.insert(0, "jepsen-etcd-demo_amd")
sys.path.insert(0, "oracle")
from test_gpu_spec import SHAPES, _finals
from lincheck import _native as N
from lincheck import history as H
from lincheck.checker import Device, Packed

shape = sys.argv[1] if len(sys.argv) > 1 else "crashed"
h = H.synth(**SHAPES[shape])
pk = Packed(h)
ref = Device(0, path_flags=N.LC_PATH_SPLIT_OFF | N.LC_PATH_SPEC_OFF).check(pk, peaks=False)
r = Device(0).check(pk, peaks=False)
big = Device(0, path_flags=N.LC_PATH_SPLIT_OFF | N.LC_PATH_SPEC_OFF, max_final=16).check(pk, peaks=False)
print("n_final hist ref", np.bincount(np.minimum(ref.n_final, 20)))
for k in range(pk.n_keys):
    a, b = _finals(r, k), _finals(ref, k)
    if a != b:
        allf = set(_finals(big, k))
        print(k, "valid", ref.valid[k], "n_final", ref.n_final[k], "big n", big.n_final[k],
              "spec in all", set(a) <= allf, "ref in all", set(b) <= allf)
        print("  spec", [(hex(x), hex(y)) for x, y in r.final[k, :4].tolist()])
        print("  ref ", [(hex(x), hex(y)) for x, y in ref.final[k, :4].tolist()])
