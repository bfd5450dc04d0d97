"""Where the drop-in's call spends its host time (bench.py --jepsen's step,
C5): cProfile of independent/checker(compose {:linear linearizable,
:timeline}) on the history, top functions by cumulative and own time."""
import cProfile
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "jepsen-etcd-demo_amd"))
import torch  # noqa: E402,F401  (the library binds torch's HIP runtime)

from lincheck import checker as CK  # noqa: E402
from lincheck import history as H  # noqa: E402
from lincheck import independent as IND  # noqa: E402
from lincheck import model as M  # noqa: E402

hist = H.synth(n_keys=1000, ops_per_key=1000, concurrency=10, anomaly_rate=0.05, seed=5)
lin = CK.linearizable({"model": M.cas_register(), "algorithm": "linear"})
chk = IND.checker(CK.compose({"linear": lin, "timeline": CK.unbridled_optimism()}))
for _ in range(3):
    chk.check({}, hist, {})
ts = []
for _ in range(10):
    t = time.perf_counter()
    chk.check({}, hist, {})
    ts.append((time.perf_counter() - t) * 1e3)
    print("call ms %.2f" % ts[-1], lin.last_timing, flush=True)
pr = cProfile.Profile()
pr.enable()
for _ in range(5):
    chk.check({}, hist, {})
pr.disable()
st = pstats.Stats(pr)
st.sort_stats("tottime").print_stats(25)
