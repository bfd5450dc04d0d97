"""Final configs without peaks (the Jepsen-shaped checkers: exact speculative
segments, k_spec<S, S, E16, EX>): segments per key 4 (the default for such
batches) against 8, device time per batch (lc_stats.kernel_ms), records
(verdicts, failing events, final-config records) required equal.
usage: python tools/ex_segs_ab.py"""
import sys

import numpy as np

sys.path.insert(0, "jepsen-etcd-demo_amd")
from lincheck import history as H  # noqa: E402
from lincheck.checker import Device, Packed  # noqa: E402

for name, cfg in [("C5", H.CONFIGS["C5"]), ("C2", H.CONFIGS["C2"]),
                  ("C5 seed 11", dict(H.CONFIGS["C5"], seed=11))]:
    pk = Packed(H.synth(**cfg))
    out = {}
    for segs in (0, 4, 8):
        dev = Device(0, spec_segs=segs)
        ms = []
        for _ in range(12):
            r = dev.check(pk, peaks=False)
            ms.append(r.stats["kernel_ms"])
        out[segs] = r
        print(f"{name:12s} spec_segs={segs or 'default'}: kernel ms median {np.median(ms[2:]):.4f} "
              f"path {r.stats['t0_path']}", flush=True)
    a = out[0]
    for segs in (4, 8):
        b = out[segs]
        diff = [f for f in ("valid", "cause", "fail_event", "n_final") if not np.array_equal(getattr(a, f), getattr(b, f))]
        # final-config records: the first n_final of each key (the rest is unwritten)
        bad = [i for i in range(len(a.valid))
               if not np.array_equal(a.final[i][:int(a.n_final[i])], b.final[i][:int(b.n_final[i])])]
        print(f"{name:12s} default vs {segs}: fields differing {diff}, keys with other final records {bad[:10]}"
              f" ({len(bad)})", flush=True)
        for i in bad[:3]:
            print("   key", i, "valid", a.valid[i], b.valid[i], "fev", a.fail_event[i], b.fail_event[i], "n_final",
                  a.n_final[i], b.n_final[i], flush=True)
            print("   a", a.final[i][:int(a.n_final[i])].tolist(), flush=True)
            print("   b", b.final[i][:int(b.n_final[i])].tolist(), flush=True)
