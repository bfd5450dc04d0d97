"""One rank of tests/test_gpu_node.py::test_two_rank_node_step (run as a
fresh process per rank, before any GPU call in it): the library's node step
(lc_check_node, one rank's context) on this rank's shard of the key space,
its block of LC_REC_* records all-gathered over gloo (the bench's host-gather
path: RCCL refuses two ranks on one GPU), rank 0 saving the node's records.
usage: node_rank_main.py RANK WORLD PORT N_KEYS OPS OUT"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "jepsen-etcd-demo_amd"), os.path.join(ROOT, "oracle")]

import numpy as np  # noqa: E402
import torch.distributed as dist  # noqa: E402  (torch first: the library binds its HIP runtime)


def main():
    rank, world, port, n_keys, ops = (int(x) for x in sys.argv[1:6])
    out = sys.argv[6]
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    from lincheck import history as H
    from lincheck import parallel as P
    from lincheck.checker import Device, Packed
    lo, hi = P.shard_range(n_keys, world, rank)
    block = -(-n_keys // world)
    h = H.synth(n_keys=hi - lo, ops_per_key=ops, concurrency=10, anomaly_rate=0.02, seed=9, key_base=lo)
    rec, st = Device(0).check_node(Packed(h), block)
    node = P.gather_blocks(np.asarray(rec, np.int64))
    if rank == 0:
        np.save(out, node)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
