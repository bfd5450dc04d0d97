"""How fast does a search started from the full config set converge to the
real one?  (Exploration for speculative key segments; CPU only.)

For a key's packed event stream and a cut event c, the run from
TOP = {(s, L) : every state s, every L within the ops pending at c} is a
superset of the real run at every later event (the search is monotone).  Once
the two sets are equal they stay equal.  Prints, over sampled keys and cuts,
how many events after the cut the sets meet (exact Knossos sets, and closed
sets as the FAST path keeps them).

    python tools/spec_conv.py [--keys 20] [--cuts 8]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "jepsen-etcd-demo_amd"))

from lincheck import history as H  # noqa: E402
from lincheck.checker import Packed  # noqa: E402

OK = 0x80000000


def step(d, s):
    f, a, b = d & 3, (d >> 2) & 0x7FFF, d >> 17
    if f == 0:
        return s
    if f == 1:
        return s if s == a else None
    if f == 2:
        return b
    return b if s == a else None


def closure(S, pend, skip=None):
    out = set(S)
    todo = list(S)
    while todo:
        s, L = todo.pop()
        for slot, d in pend.items():
            if slot == skip or slot in L:
                continue
            t = step(d, s)
            if t is None:
                continue
            c = (t, L | frozenset([slot]))
            if c not in out:
                out.add(c)
                todo.append(c)
    return out


def ok_exact(S, pend, p):
    ret = {(s, L - {p}) for (s, L) in S if p in L}
    I = closure({(s, L) for (s, L) in S if p not in L}, pend, skip=p)
    d = pend[p]
    for s, L in I:
        t = step(d, s)
        if t is not None:
            ret.add((t, L))
    return ret


def ok_closed(S, pend, p):
    C = closure(S, pend)
    return {(s, L - {p}) for (s, L) in C if p in L}


def run(events, desc, c, S, pend, okf, limit):
    """Yield the config set after every event from c on (up to limit)."""
    pend = dict(pend)
    for j in range(c, min(len(events), c + limit)):
        w = int(events[j])
        slot = (w >> 24) & 0x7F
        if w & OK:
            S = okf(S, pend, slot)
            del pend[slot]
        else:
            pend[slot] = desc[w & 0xFFFFFF]
        yield j, S, pend


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--keys", type=int, default=20)
    ap.add_argument("--cuts", type=int, default=8)
    ap.add_argument("--ops", type=int, default=1000)
    ap.add_argument("--think", type=float, default=1.0)
    ap.add_argument("--limit", type=int, default=400)
    args = ap.parse_args()
    h = H.synth(n_keys=args.keys, ops_per_key=args.ops, concurrency=10, seed=2, mean_think=args.think)
    pk = Packed(h)
    rng = np.random.default_rng(0)
    for mode, okf in (("closed", ok_closed), ("exact", ok_exact)):
        meets, pends = [], []
        for k in range(pk.n_keys):
            ev = pk.events(k)
            n = len(ev)
            desc = {}
            for w in ev:
                w = int(w)
                if not w & OK:
                    t = w & 0xFFFFFF
                    desc[t] = pk.desc(k, t)
            states = set()
            for d in desc.values():
                states.add((d >> 2) & 0x7FFF if (d & 3) in (1, 3) else 0)
                if (d & 3) >= 2:
                    states.add(d >> 17)
            states.add(0)
            # the real run, recording sets and pending ops at every event
            real = [None] * n
            S, pend = {(0, frozenset())}, {}
            for j, S, pend in run(ev, desc, 0, S, pend, okf, n):
                real[j] = (S, dict(pend))
            for c in sorted(rng.choice(np.arange(n // 8, n - args.limit), args.cuts, replace=False)):
                S_c, pend_c = real[c - 1]
                subsets = [frozenset()]
                for slot in pend_c:
                    subsets += [L | {slot} for L in subsets]
                top = {(s, L) for s in states for L in subsets}
                pends.append(len(pend_c))
                met = None
                for j, T, _ in run(ev, desc, c, top, pend_c, okf, args.limit):
                    if T == real[j][0]:
                        met = j - c + 1
                        break
                meets.append(met if met is not None else 10 ** 9)
        m = np.array(meets)
        print(f"{mode}: cuts {len(m)}, pending at cut mean {np.mean(pends):.1f}; events to meet: "
              f"median {np.median(m):.0f}, p90 {np.percentile(m, 90):.0f}, max {m.max()}, "
              f"never (>{args.limit}) {(m >= 10 ** 9).sum()}")


if __name__ == "__main__":
    main()
