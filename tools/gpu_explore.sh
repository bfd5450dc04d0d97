# Exploration pass: k_spec phase stamps at 4 / 6 / 8 segments per key (C2),
# register-tier A/B on a C3 shard, and the N = 2 rehearsal with the default
# (RCCL) gather, which RCCL refuses on one device: the bench must fall back to gloo.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/explore
mkdir -p $O
echo "== stamps $(date +%T)"
for S in 4 6 8; do
LINCHECK_LIB_OVERRIDE=$PWD/jepsen-etcd-demo_amd/lincheck/liblincheck_specst.so timeout -k 10 300 python -u tools/spec_stamps.py 1000 $S 0 $O/st$S.npz > $O/st$S.txt 2>&1 || { tail -5 $O/st$S.txt; exit 1; }
head -14 $O/st$S.txt
done
echo "== c3 shard ab $(date +%T)"
timeout -k 10 300 python -u tools/spec_ab.py C3 12500 2000 default spec_segs=2 spec_segs=4 > $O/ab_c3s.txt 2>&1 || { tail -5 $O/ab_c3s.txt; exit 1; }
cat $O/ab_c3s.txt
echo "== n2 rccl-fallback rehearsal $(date +%T)"
LC_BENCH_DEVICE=0 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --keys 20000 --steps 5 --warmup 1 > $O/n2.json 2> $O/n2.err || { tail -20 $O/n2.err; exit 1; }
cut -c1-600 $O/n2.json
grep -i rccl $O/n2.err | head -5
echo ALL_OK
