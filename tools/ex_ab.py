"""Final configs without peaks (the Knossos-shaped checkers): exact speculative
segments vs the unsegmented exact search, device time per batch (lc_stats.kernel_ms)."""
import sys
import numpy as np
sys.path.insert(0, "jepsen-etcd-demo_amd")
from lincheck import _native as N
from lincheck import history as H
from lincheck.checker import Device, Packed

for name, kw in [("C2 1000x1000", dict(n_keys=1000, ops_per_key=1000, concurrency=10, seed=7)),
                 ("C5 1000x1000", dict(n_keys=1000, ops_per_key=1000, concurrency=10, anomaly_rate=0.05, seed=8)),
                 ("C3 12500x2000", dict(n_keys=12500, ops_per_key=2000, concurrency=10, seed=9))]:
    pk = Packed(H.synth(**kw))
    out = {}
    for lab, dev in [("exact spec", Device(0)), ("unsegmented", Device(0, path_flags=N.LC_PATH_SPEC_OFF)),
                     ("verdicts", Device(0))]:
        ms = []
        for i in range(6):
            r = dev.check(pk, verdicts_only=(lab == "verdicts"), peaks=False)
            ms.append(r.stats["kernel_ms"])
        out[lab] = r
        print(f"{name:16s} {lab:12s} kernel ms {np.round(ms[1:], 3)} median {np.median(ms[1:]):.3f} "
              f"path {r.stats['t0_path']}", flush=True)
    a, b = out["exact spec"], out["unsegmented"]
    same = all((getattr(a, f) == getattr(b, f)).all() for f in ("valid", "cause", "fail_event", "n_final"))
    print(f"{name:16s} same {same}", flush=True)
