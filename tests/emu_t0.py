"""Lane-level CPU model of the register-lattice tier (device_lattice.hip, T0).

Test infrastructure: it re-executes the kernel's per-event steps on 64-lane
numpy arrays -- the one-directional DPP / permlane gathers (with garbage on
the lanes a gather does not define, so a missing mask shows up), the
lane-masked transfer masks, the Gauss-Seidel closure sweeps and the
two-step relocation -- so the algorithm can be checked against the oracle
without a GPU.  It never stands in for the device: tests compare both
against the oracle separately.
"""
from __future__ import annotations

import numpy as np

LANES = np.arange(64, dtype=np.int64)
OK_BIT = 0x80000000
RNG = np.random.default_rng(12345)


def garbage():
    return RNG.integers(0, 2**32, 64, dtype=np.uint64).astype(np.uint32)


def gdown(x, q):
    """x[L - 2^q] on lanes with bit q; garbage elsewhere."""
    out = garbage()
    has = (LANES >> q) & 1 == 1
    out[has] = x[LANES[has] - (1 << q)]
    return out


def gup(x, q):
    """x[L + 2^q] on lanes without bit q; garbage elsewhere."""
    out = garbage()
    no = (LANES >> q) & 1 == 0
    out[no] = x[LANES[no] + (1 << q)]
    return out


def umin1(t):
    return np.minimum(t, 1).astype(np.uint32)


def xacc(acc, x, pas, keep, b):
    acc = (x & pas) | acc
    return ((umin1(x & keep) << np.uint32(b)) | acc).astype(np.uint32)


def xfer_of(d):
    f, a, b = d & 3, (d >> 2) & 0x7FFF, d >> 17
    abit = (1 << a) if a < 32 else 0
    pas = 0xFFFFFFFF if f == 0 else (abit if f == 1 else 0)
    keep = 0xFFFFFFFF if f == 2 else (abit if f == 3 else 0)
    bb = (b & 31) if f >= 2 else 0
    return pas, keep, bb


class Ops:
    """Per dense index: (pass, keep, b) -- the lanes of pass_v / keep_v / b_v."""

    def __init__(self):
        self.pas = [0] * 64
        self.keep = [0] * 64
        self.b = [0] * 64


def lane_masks(ops, N, p):
    vp, vk = [], []
    for q in range(min(N, 6)):
        on = ((LANES >> q) & 1 == 1) & (q != p)
        vp.append(np.where(on, np.uint32(ops.pas[q]), np.uint32(0)).astype(np.uint32))
        vk.append(np.where(on, np.uint32(ops.keep[q]), np.uint32(0)).astype(np.uint32))
    sb = [ops.b[q] for q in range(N)]
    return vp, vk, sb


def sweep_lanes(cur, vp, vk, sb, N):
    for q in range(min(N, 6)):
        x = gdown(cur, q)
        cur = xacc(cur, x, vp[q], vk[q], sb[q])
    return cur


def ok_lane(W0, p, live, ops):
    """ok_lane: every live index < 6, lowest-free indices, no relocation."""
    cand = live & ~(1 << p)
    vp, vk = [], []
    for q in range(6):
        on = ((LANES >> q) & 1 == 1) & bool((cand >> q) & 1)
        vp.append(np.where(on, np.uint32(ops.pas[q]), np.uint32(0)).astype(np.uint32))
        vk.append(np.where(on, np.uint32(ops.keep[q]), np.uint32(0)).astype(np.uint32))
    sb = [ops.b[q] for q in range(6)]
    hp = (LANES >> p) & 1 == 1
    Ret = np.where(hp, 0, gup(W0, p)).astype(np.uint32)
    I = np.where(hp, 0, W0).astype(np.uint32)
    for _s in range(bin(cand).count("1")):
        nv = sweep_lanes(I, vp, vk, sb, 6)
        ch = (nv != I).any()
        I = nv
        if not ch:
            break
    Ret = xacc(Ret, I, ops.pas[p], ops.keep[p], ops.b[p])
    if not Ret.any():
        return 1, W0
    return 0, Ret


def ok_event(W, p, n, ops):
    """One :ok(p) with n pending; W = list of RL lane arrays. Returns (status, W')."""
    RL = 1 if n <= 6 else 1 << (n - 6)
    NB = n
    NR = max(0, NB - 6)
    vp, vk, sb = lane_masks(ops, NB, p)
    rp = [ops.pas[6 + r] if 6 + r != p else 0 for r in range(NR)]
    rk = [ops.keep[6 + r] if 6 + r != p else 0 for r in range(NR)]
    pp, pk, pb = ops.pas[p], ops.keep[p], ops.b[p]
    Ret, I = [None] * RL, [None] * RL
    if p < 6:
        hp = (LANES >> p) & 1 == 1
        for k in range(RL):
            u = gup(W[k], p)
            Ret[k] = np.where(hp, 0, u).astype(np.uint32)
            I[k] = np.where(hp, 0, W[k]).astype(np.uint32)
    else:
        r = p - 6
        for k in range(RL):
            hk = (k >> r) & 1
            Ret[k] = np.zeros(64, np.uint32) if hk else W[k | (1 << r)].copy()
            I[k] = np.zeros(64, np.uint32) if hk else W[k].copy()
    for _s in range(1, NB):
        nv = [sweep_lanes(I[k], vp, vk, sb, NB) for k in range(RL)]
        for r in range(NR):
            for k in range(RL):
                if (k >> r) & 1:
                    nv[k] = xacc(nv[k], nv[k ^ (1 << r)], rp[r], rk[r], sb[6 + r])
        ch = any((nv[k] != I[k]).any() for k in range(RL))
        I = nv
        if not ch:
            break
    for k in range(RL):
        Ret[k] = xacc(Ret[k], I[k], pp, pk, pb)
    if not any(Ret[k].any() for k in range(RL)):
        return 1, W
    last = n - 1
    if p == last:
        return 0, Ret
    Wn = [None] * RL
    if last < 6:  # single register
        z = gdown(gup(Ret[0], last), p)
        hl = (LANES >> last) & 1 == 1
        hp = (LANES >> p) & 1 == 1
        Wn[0] = np.where(hl, 0, np.where(hp, z, Ret[0])).astype(np.uint32)
        return 0, Wn
    rl = NR - 1
    for k in range(RL):
        if (k >> rl) & 1:
            Wn[k] = np.zeros(64, np.uint32)
            continue
        if p < 6:
            hp = (LANES >> p) & 1 == 1
            z = gdown(Ret[k | (1 << rl)], p)
            Wn[k] = np.where(hp, z, Ret[k]).astype(np.uint32)
        else:
            r = p - 6
            Wn[k] = Ret[(k ^ (1 << r)) | (1 << rl)].copy() if (k >> r) & 1 else Ret[k].copy()
    return 0, Wn


def xv(x, q):
    """x[L ^ 2^q] (both directions)."""
    return x[LANES ^ (1 << q)]


def xapply(M, pas, keep, st):
    return ((M & np.uint32(pas)) | np.where((M & np.uint32(keep)) != 0, np.uint32(st), np.uint32(0))).astype(np.uint32)


def ok_event_mem(Wm, p, n, ops):
    """ok_event_mem<RL>: the workspace path for 9-10 pending (in-place sweeps)."""
    RL = 1 << (n - 6)
    NB = n
    cand = ((1 << n) - 1) & ~(1 << p)
    PS = [ops.pas[q] if (cand >> q) & 1 else 0 for q in range(NB)]
    KP = [ops.keep[q] if (cand >> q) & 1 else 0 for q in range(NB)]
    ST = [1 << ops.b[q] for q in range(NB)]
    pp, pk, pt = ops.pas[p], ops.keep[p], 1 << ops.b[p]
    plm = (1 << p) if p < 6 else 0
    prm = (1 << (p - 6)) if p >= 6 else 0
    R = [None] * RL
    I = [None] * RL
    for k in range(RL):
        w = Wm[k]
        src = Wm[k ^ prm][LANES ^ plm]
        hp = ((LANES & plm) != 0) | bool(k & prm)
        R[k] = np.where(hp, 0, src).astype(np.uint32)
        I[k] = np.where(hp, 0, w).astype(np.uint32)
    while True:
        ch = False
        for k in range(RL):
            x = I[k].copy()
            acc = x.copy()
            for q in range(6):
                y = xv(x, q)
                acc |= np.where((LANES >> q) & 1 == 1, xapply(y, PS[q], KP[q], ST[q]), 0).astype(np.uint32)
            for q in range(6, NB):
                if (k >> (q - 6)) & 1:
                    acc |= xapply(I[k ^ (1 << (q - 6))], PS[q], KP[q], ST[q])
            if (acc != x).any():
                I[k] = acc
                ch = True
        if not ch:
            break
    cS = 0
    for k in range(RL):
        R[k] = R[k] | xapply(I[k], pp, pk, pt)
        cS += int(np.count_nonzero(R[k]))
    if cS == 0:
        return 1, Wm
    last = n - 1
    llm = (1 << last) if last < 6 else 0
    lrm = (1 << (last - 6)) if last >= 6 else 0
    Wn = [None] * RL
    for k in range(RL):
        r = R[k]
        src = R[k ^ (prm | lrm)][LANES ^ (plm | llm)]
        hp = ((LANES & plm) != 0) | bool(k & prm)
        hl = ((LANES & llm) != 0) | bool(k & lrm)
        Wn[k] = r.copy() if p == last else np.where(hl, 0, np.where(hp, src, r)).astype(np.uint32)
    return 0, Wn


def ok_lane_closed(W0, p, live, ops, dirty):
    """ok_lane_closed: close W under every live op (p included), then keep the
    lanes with bit p, shifted down (the fast path's closed-set invariant)."""
    C = W0
    if dirty:
        vp, vk = [], []
        for q in range(6):
            on = ((LANES >> q) & 1 == 1) & bool((live >> q) & 1)
            vp.append(np.where(on, np.uint32(ops.pas[q]), np.uint32(0)).astype(np.uint32))
            vk.append(np.where(on, np.uint32(ops.keep[q]), np.uint32(0)).astype(np.uint32))
        sb = [ops.b[q] for q in range(6)]
        for _s in range(bin(live).count("1")):
            nv = sweep_lanes(C, vp, vk, sb, 6)
            ch = (nv != C).any()
            C = nv
            if not ch:
                break
    hp = (LANES >> p) & 1 == 1
    Wn = np.where(hp, 0, gup(C, p)).astype(np.uint32)
    if not Wn.any():
        return 1, W0
    return 0, Wn


def check_key(events, trans, tb=0, init_state=0, closed=False):
    """Model of lattice_key: returns (valid, fail_event) or None (spill).
    closed: the fast path's lane phase (closed sets, ok_lane_closed)."""
    W = [np.zeros(64, np.uint32) for _ in range(16)]
    W[0][0] = 1 << init_state
    ops = Ops()
    slot_v = [0] * 64
    dense = [0] * 128
    n = 0
    live = 0
    dirty = True
    for j, ev in enumerate(events):
        ev = int(ev)
        slot = (ev >> 24) & 0x7F
        if not ev & OK_BIT:
            if n >= 10 or slot >= 64:
                return None
            pas, keep, b = xfer_of(int(trans[tb + (ev & 0xFFFFFF)]))
            idx = (~live & -~live).bit_length() - 1
            ops.pas[idx], ops.keep[idx], ops.b[idx] = pas, keep, b
            slot_v[idx] = slot
            dense[slot] = idx
            live |= 1 << idx
            n += 1
            dirty = True
            continue
        p = dense[slot]
        if n <= 6:
            if closed:
                st, W0 = ok_lane_closed(W[0], p, live, ops, dirty)
                dirty = False
            else:
                st, W0 = ok_lane(W[0], p, live, ops)
            if st == 1:
                return 0, j
            W[0] = W0
            live &= ~(1 << p)
            n -= 1
            continue
        RL = 1 if n <= 6 else 1 << (n - 6)
        st, Wn = (ok_event_mem if n >= 9 else ok_event)(W[:RL], p, n, ops)
        if st == 1:
            return 0, j
        for k in range(RL):
            W[k] = Wn[k]
        last = n - 1
        if p != last:
            s_last = slot_v[last]
            ops.pas[p], ops.keep[p], ops.b[p] = ops.pas[last], ops.keep[last], ops.b[last]
            slot_v[p] = s_last
            dense[s_last] = p
        n -= 1
        live = (1 << n) - 1
        dirty = True  # the dense phase keeps exact sets
    return 1, -1
