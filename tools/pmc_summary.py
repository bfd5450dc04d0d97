"""Sum rocprofv3 PMC counters per kernel over the last dispatch of each kernel (sqlite output)."""
import sqlite3, sys, glob, collections
for f in sys.argv[1:]:
    c = sqlite3.connect(f)
    rows = c.execute("select dispatch_id, kernel_name, counter_name, value from counters_collection").fetchall()
    last = {}
    for d, k, n, v in rows:
        last.setdefault(k, {})
        last[k].setdefault(d, collections.defaultdict(float))[n] += v
    for k, ds in last.items():
        if "lattice" not in k and len(sys.argv) < 3: pass
        d = max(ds)
        print(f, k[:60], dict(ds[d]))
