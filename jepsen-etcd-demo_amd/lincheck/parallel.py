"""Key sharding across GPUs and the one exchange step of the path.

jepsen.independent/checker runs its per-key checks in a bounded pmap on one
JVM (etcdemo.clj:115); keys share no state.  Here keys
are split over ranks (one process per GPU), each rank searches its shard,
and the fixed-size per-key verdict records are all-gathered -- over RCCL
(torch.distributed "nccl") on MI355X, over gloo in CPU tests.

Record (int64): bits 0..7 valid+1, 8..15 cause, 16..47 failing event + 1
(include/lincheck.h LC_REC_*; 0 = padding).  A node step (lc_check_node)
lays the records out in blocks of `block` per rank, each rank's shard first
in its block and the rest padded with 0, blocks in rank order.
"""

from __future__ import annotations

from typing import List, Sequence, Tuple

import numpy as np


def shard_range(n_keys: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous balanced shard [lo, hi) of n_keys equal-cost keys."""
    q, r = divmod(n_keys, world)
    lo = rank * q + min(rank, r)
    return lo, lo + q + (1 if rank < r else 0)


def lpt_shards(costs: Sequence[float], world: int) -> List[np.ndarray]:
    """Longest-processing-time-first assignment of keys to ranks."""
    costs = np.asarray(costs, dtype=np.float64)
    order = np.argsort(-costs, kind="stable")
    load = np.zeros(world)
    out: List[List[int]] = [[] for _ in range(world)]
    for k in order:
        r = int(np.argmin(load))
        out[r].append(int(k))
        load[r] += costs[k]
    return [np.array(sorted(x), dtype=np.int64) for x in out]


def key_costs(hist, budget: int = 1 << 20) -> Tuple[np.ndarray, np.ndarray]:
    """SURVEY.md 8(e) E-1's cost estimate per key, from the history's columns
    alone (before anything is packed): ops x concurrency x 2^crashed, with
    2^crashed capped at the search budget (a key's config sets never exceed
    it).  ops = the key's rows / 2, concurrency = its distinct processes,
    crashed = its :info completions (ops callable forever: each can double the
    frontier).  Returns (keys in order of first appearance -- the packed
    batch's key order -- and their costs)."""
    from . import _native as N
    key = np.asarray(hist.key, np.int64)
    has = key != N.LC_NO_KEY
    rows = np.flatnonzero(has)
    keys, first, inv, n_rows = np.unique(key[rows], return_index=True, return_inverse=True, return_counts=True)
    order = np.argsort(first, kind="stable")          # first appearance
    info = np.bincount(inv, weights=(np.asarray(hist.type)[rows] == N.LC_INFO), minlength=keys.size)
    kp = np.unique(np.stack([inv, np.asarray(hist.process, np.int64)[rows]]), axis=1)
    procs = np.bincount(kp[0], minlength=keys.size)
    cap = max(0, int(budget).bit_length() - 1)
    cost = (n_rows / 2.0) * np.maximum(procs, 1) * np.exp2(np.minimum(info, cap))
    return keys[order], cost[order]


def cost_shards(costs: Sequence[float], world: int, heavy: float = 1.0 / 32) -> List[np.ndarray]:
    """Key indices of each rank (sorted), balanced by estimated cost (E-1).

    Keys costing more than `heavy` of one rank's fair share go first, by LPT
    (longest first, each to the least-loaded rank): those are the keys that
    would otherwise leave one rank holding the walk that decides the node's
    time.  The rest, in key order, are then cut into one contiguous run per
    rank, sized by water-filling so every rank ends as near the common level
    as whole keys allow (each rank's load is within one light key -- at most
    `heavy` of a share -- of it, unless its heavy keys alone exceed it).
    With equal costs there are no heavy keys and the shards are contiguous
    balanced ranges, as shard_range's (the bench synthesises a rank's range
    directly)."""
    costs = np.asarray(costs, dtype=np.float64)
    n = costs.size
    if world <= 1 or n == 0:
        return [np.arange(n, dtype=np.int64)] + [np.zeros(0, np.int64) for _ in range(max(world, 1) - 1)]
    total = float(costs.sum())
    thr = heavy * total / world
    is_heavy = costs > thr
    load = np.zeros(world)
    parts: List[List[int]] = [[] for _ in range(world)]
    hv = np.flatnonzero(is_heavy)
    for k in hv[np.argsort(-costs[hv], kind="stable")]:
        r = int(np.argmin(load))
        parts[r].append(int(k))
        load[r] += costs[k]
    light = np.flatnonzero(~is_heavy)
    lt = float(costs[light].sum())
    # water level lam: sum over ranks of max(0, lam - load) = lt
    srt = np.sort(load)
    lam = srt[-1]
    for i in range(world):
        # level between srt[i] and srt[i+1] fills the i+1 lowest ranks
        nxt = srt[i + 1] if i + 1 < world else np.inf
        need = (i + 1) * nxt - srt[:i + 1].sum()
        if need >= lt:
            lam = (lt + srt[:i + 1].sum()) / (i + 1)
            break
    quota = np.maximum(0.0, lam - load)
    bounds = np.cumsum(quota)
    cum = np.cumsum(costs[light])
    mid = cum - costs[light] / 2.0
    owner = np.minimum(np.searchsorted(bounds, mid, side="left"), world - 1)
    return [np.sort(np.concatenate([np.asarray(parts[r], np.int64), light[owner == r]])) for r in range(world)]


def shard_costs(costs: Sequence[float], shards: Sequence[np.ndarray]) -> np.ndarray:
    """Each rank's estimated cost under a sharding."""
    costs = np.asarray(costs, dtype=np.float64)
    return np.array([costs[s].sum() for s in shards])


def contiguous(shard: np.ndarray) -> bool:
    """Whether a shard is one run of consecutive key indices."""
    return shard.size == 0 or int(shard[-1]) - int(shard[0]) + 1 == shard.size


def node_key_order(node, shards: Sequence[np.ndarray], block: int):
    """(valid, cause, fail_event) of every key in the caller's key order from
    the gathered node records (rank r's records are the first len(shards[r])
    of block r, in the order of shards[r]; the padding must be 0)."""
    v, c, fe = node_verdicts(node, [len(s) for s in shards], block)
    n = sum(len(s) for s in shards)
    at = np.concatenate([np.asarray(s, np.int64) for s in shards]) if shards else np.zeros(0, np.int64)
    if n and not np.array_equal(np.sort(at), np.arange(n)):
        raise ValueError("shards do not partition the keys")
    vo, co, fo = np.empty_like(v), np.empty_like(c), np.empty_like(fe)
    vo[at], co[at], fo[at] = v, c, fe
    return vo, co, fo


def pack_records(valid, cause, fail_event):
    """Verdict records, numpy or torch (same arithmetic)."""
    try:
        import torch
        if isinstance(valid, torch.Tensor):
            return ((fail_event.to(torch.int64) + 1) << 16) | (cause.to(torch.int64) << 8) | (valid.to(torch.int64) + 1)
    except ImportError:
        pass
    return ((np.asarray(fail_event, np.int64) + 1) << 16) | (np.asarray(cause, np.int64) << 8) | \
        (np.asarray(valid, np.int64) + 1)


def unpack_records(rec: np.ndarray):
    rec = np.asarray(rec, dtype=np.int64)
    valid = ((rec & 0xFF) - 1).astype(np.int8)
    cause = ((rec >> 8) & 0xFF).astype(np.uint8)
    fail_event = ((rec >> 16) - 1).astype(np.int32)
    return valid, cause, fail_event


def gather_records(keys, records, group=None):
    """All-gather (key, record) pairs of every rank; shards may differ in size.

    keys / records: 1-D int64 torch tensors on the backend's device.
    Returns numpy (keys, records) of all ranks, in rank order.
    """
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    n = torch.tensor([keys.numel()], dtype=torch.int64, device=keys.device)
    sizes = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(sizes, n, group=group)
    m = int(max(int(s.item()) for s in sizes))
    pad = torch.full((2, m), -1, dtype=torch.int64, device=keys.device)
    pad[0, :keys.numel()] = keys
    pad[1, :keys.numel()] = records
    out = torch.empty(world * 2 * m, dtype=torch.int64, device=keys.device)
    dist.all_gather_into_tensor(out, pad.reshape(-1), group=group)
    out = out.cpu().numpy().reshape(world, 2, m)
    ks, rs = [], []
    for r in range(world):
        c = int(sizes[r].item())
        ks.append(out[r, 0, :c]); rs.append(out[r, 1, :c])
    return np.concatenate(ks), np.concatenate(rs)


def node_block(valid, cause, fail_event, block: int) -> np.ndarray:
    """This rank's block of node records as lc_check_node lays it out: the
    shard's records, padded with 0 (never a record: an :unknown key, the one
    whose valid + 1 is 0, always has a cause, LC_CAUSE_BUDGET or above)."""
    rec = np.asarray(pack_records(valid, cause, fail_event), np.int64)
    if rec.size > block:
        raise ValueError(f"a shard of {rec.size} keys does not fit a block of {block}")
    out = np.zeros(block, np.int64)
    out[:rec.size] = rec
    return out


def gather_blocks(block_rec, group=None) -> np.ndarray:
    """All-gather every rank's equal-size block in rank order: what
    lc_check_node's ncclAllGather does over RCCL, here over the process
    group's backend (gloo on the host)."""
    import torch
    import torch.distributed as dist
    t = torch.from_numpy(np.ascontiguousarray(block_rec, dtype=np.int64))
    world = dist.get_world_size(group)
    out = torch.empty(world * t.numel(), dtype=torch.int64)
    dist.all_gather_into_tensor(out, t, group=group)
    return out.numpy()


def node_verdicts(node, shard_sizes: Sequence[int], block: int):
    """Per-key (valid, cause, fail_event) of the node's key space, in key
    order, from the gathered blocks: rank r's shard is the first
    shard_sizes[r] records of block r.  The padding must be all 0."""
    node = np.asarray(node, np.int64)
    if node.size < block * len(shard_sizes):
        raise ValueError("node records shorter than the blocks")
    parts = []
    for r, n in enumerate(shard_sizes):
        blk = node[r * block:(r + 1) * block]
        if (blk[n:] != 0).any():
            raise ValueError(f"rank {r}'s block has records past its shard")
        parts.append(blk[:n])
    return unpack_records(np.concatenate(parts) if parts else np.zeros(0, np.int64))
