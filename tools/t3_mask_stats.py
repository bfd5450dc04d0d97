"""Diagnostic (not a test): how many distinct linearized-sets L a C4 key's
config sets hold against their configs -- the case for keying T3's hash sets
by L with a state bitmask per entry.  Pure-Python search over the packed
stream of a few keys (same sets as every tier).
usage: python tools/t3_mask_stats.py [keys] [budget]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "jepsen-etcd-demo_amd"))

from lincheck import history as H  # noqa: E402
from lincheck.checker import Packed  # noqa: E402

LM = (1 << 56) - 1


def step(s, d):
    f, a, b = d & 3, (d >> 2) & 0x7FFF, d >> 17
    ok = f == 0 or f == 2 or s == a
    return ok, (b if f >= 2 else s)


def run(p, k, budget):
    ev = p.events(k)
    slot_desc = {}
    pend = set()
    S = {0}
    tot = dict(oks=0, cfgS=0, entS=0, cfgI=0, entI=0, maxlayer=0, big=0)
    for i, w in enumerate(ev):
        w = int(w)
        slot = (w >> 24) & 0x7F
        if not (w >> 31):
            slot_desc[slot] = p.desc(k, w & 0xFFFFFF)
            pend.add(slot)
            continue
        pp = slot
        Sn = set()
        I = set()
        for c in S:
            if (c >> pp) & 1:
                Sn.add(c & ~(1 << pp))
            else:
                I.add(c)
        front = list(I)
        layers = {}
        while front:
            nf = []
            for c in front:
                st = c >> 56
                for q in pend:
                    if q == pp or (c >> q) & 1:
                        continue
                    ok, s2 = step(st, slot_desc[q])
                    if ok:
                        c2 = (s2 << 56) | (c & LM) | (1 << q)
                        if c2 not in I:
                            I.add(c2)
                            nf.append(c2)
            front = nf
            if len(I) > budget:
                return tot, i
        for c in I:
            ok, s2 = step(c >> 56, slot_desc[pp])
            if ok:
                Sn.add((s2 << 56) | (c & LM))
        if not Sn or len(Sn) > budget:
            return tot, i
        for c in I:
            layers.setdefault(bin(c & LM).count("1"), set()).add(c & LM)
        tot["oks"] += 1
        tot["cfgS"] += len(S)
        tot["entS"] += len({c & LM for c in S})
        tot["cfgI"] += len(I)
        tot["entI"] += len({c & LM for c in I})
        if len(I) > 2048:
            tot["big"] += 1
            tot["maxlayer"] = max(tot["maxlayer"], max(len(v) for v in layers.values()))
        S = Sn
        pend.discard(pp)
    return tot, len(ev)


def main():
    nk = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    budget = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 16
    h = H.synth(**dict(H.CONFIGS["C4"], n_keys=nk))
    p = Packed(h)
    for k in range(nk):
        tot, end = run(p, k, budget)
        print(f"key {k}: ended at event {end}/{p.n_events(k)}; {tot}; "
              f"configs per L: S {tot['cfgS'] / max(1, tot['entS']):.2f}, I {tot['cfgI'] / max(1, tot['entI']):.2f}")


if __name__ == "__main__":
    main()
