"""One rank of tests/test_gpu_node.py::test_two_rank_node_step (run as a
fresh process per rank, before any GPU call in it): the library's node step
(lc_check_node, one rank's context) on this rank's cost-balanced shard of a
mixed key space (parallel.key_costs / cost_shards, SURVEY E-1),
its block of LC_REC_* records all-gathered over gloo (the bench's host-gather
path: RCCL refuses two ranks on one GPU), rank 0 saving the node's records.
usage: node_rank_main.py RANK WORLD PORT N_KEYS OPS OUT"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "jepsen-etcd-demo_amd"), os.path.join(ROOT, "oracle")]

import numpy as np  # noqa: E402
import torch.distributed as dist  # noqa: E402  (torch first: the library binds its HIP runtime)


BUDGET = 1 << 16


def mixed_history(n_keys, ops):
    """n_keys C2/C5-shaped keys (concurrency 10, 2 % anomalous) followed by 6
    C4-shaped ones (concurrency 30, 2 % crashed write/cas): the batch whose
    contiguous split leaves every C4-shaped key on the last rank."""
    from lincheck import history as H
    return H.History.concat([
        H.synth(n_keys=n_keys, ops_per_key=ops, concurrency=10, anomaly_rate=0.02, seed=9),
        H.synth(n_keys=6, ops_per_key=400, concurrency=30, info_rate=0.02, seed=4, key_base=n_keys)])


def main():
    rank, world, port, n_keys, ops = (int(x) for x in sys.argv[1:6])
    out = sys.argv[6]
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    from lincheck import history as H
    from lincheck import parallel as P
    from lincheck.checker import Device, Packed
    h = mixed_history(n_keys, ops)
    keys, costs = P.key_costs(h, BUDGET)
    shards = P.cost_shards(costs, world)
    block = max(len(s) for s in shards)
    rec, st = Device(0, budget=BUDGET).check_node(Packed(h.select_keys(keys[shards[rank]])), block)
    node = P.gather_blocks(np.asarray(rec, np.int64))
    if rank == 0:
        np.save(out, node)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
