"""Phase cycles of the device WGL walk (the LC_WGL_PROF build:
make -C jepsen-etcd-demo_amd variant NAME=wglprof VFLAGS=-DLC_WGL_PROF).
usage: LINCHECK_LIB_OVERRIDE=jepsen-etcd-demo_amd/lincheck/liblincheck_wglprof.so \\
       python tools/wgl_prof.py [C2|C4|C5] [budget]
Prints each phase's s_memtime cycles summed over the keys, per step."""
import ctypes as C
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "jepsen-etcd-demo_amd"))
from lincheck import _native as N  # noqa: E402
from lincheck import checker as CK  # noqa: E402
from lincheck import history as H  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "C2"
budget = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 20
hist = H.synth(**H.CONFIGS[cfg]) if cfg in H.CONFIGS else H.synth(n_keys=1000, ops_per_key=1000, seed=5,
                                                                    anomaly_rate=0.05)
packed = CK.Packed(hist)
dev = CK.Device(0, budget=budget, algorithm=N.LC_ALGO_WGL)
fn = N.lib().lc_debug_wgl_prof
fn.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
buf = (C.c_ulonglong * 8)()
res = dev.check(packed, verdicts_only=True)  # warm-up (tables, code)
fn(buf, 1)
res = dev.check(packed, verdicts_only=True)
fn(buf, 1)
v = list(buf)
steps = max(v[7], 1)
names = ["staging", "probe rounds", "child scans", "backtracks", "steps down", "advances", "probe iterations",
         "steps down (count)"]
out = {"config": cfg, "budget": budget, "wgl_ms": res.stats["wgl_ms"], "wgl_steps": res.stats["wgl_steps"],
       "keys": packed.n_keys, "valid": int((res.valid == 1).sum()), "unknown": int((res.valid == -1).sum()),
       "phases": {names[i]: v[i] for i in range(8)},
       "cycles_per_step_down": {names[i]: round(v[i] / steps, 1) for i in range(6)}}
print(json.dumps(out))
