# Layered-tier A/B on C4 (2^16 budget): the product build against variants.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/t3ab
mkdir -p $O
timeout -k 10 200 python -u tools/t3_ab.py 65536 5 2>&1 | tee -a $O/ab.txt || exit 1
for v in ${VARIANTS:-t3rb}; do
LINCHECK_LIB_OVERRIDE=$PWD/jepsen-etcd-demo_amd/lincheck/liblincheck_$v.so timeout -k 10 200 python -u tools/t3_ab.py 65536 5 2>&1 | tee -a $O/ab.txt || exit 1
done
echo T3AB_OK
