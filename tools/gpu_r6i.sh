# Round 6: rehearsal of bench.py's N > 1 path (cost-balanced shards, records
# back in key order) on the one GPU: every rank on cuda:0, records gathered on
# the host (LC_BENCH_GATHER=host), 2 and 3 ranks (uneven shards).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6i; mkdir -p $O
export LC_BENCH_GATHER=host LC_BENCH_DEVICE=0
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 \
  bench.py --gpus 2 --steps 5 --warmup 2 --keys 20001 > $O/n2.json 2> $O/n2.err || { tail -20 $O/n2.err; exit 1; }
cut -c1-400 $O/n2.json
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 3 --master-addr 127.0.0.1 --master-port 29512 \
  bench.py --gpus 3 --steps 5 --warmup 2 --keys 9001 > $O/n3.json 2> $O/n3.err || { tail -20 $O/n3.err; exit 1; }
cut -c1-400 $O/n3.json
