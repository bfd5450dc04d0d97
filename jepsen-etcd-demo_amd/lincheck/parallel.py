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
