# Speculative checkpoints: first checkpoint at 16 / 24 events past a cut
# against the default 32 (spec_ck = (ck1 + 1) | (ck2 + 1) << 16).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/ck
mkdir -p $O
S="default spec_ck=0x790011 spec_ck=0x790019 spec_ck=0x510011"
timeout -k 10 200 python -u tools/spec_ab.py C2 1000 1000 $S 2>&1 | tee $O/ab_c2.txt || exit 1
timeout -k 10 200 python -u tools/spec_ab.py C5 1000 1000 $S 2>&1 | tee $O/ab_c5.txt || exit 1
timeout -k 10 200 python -u tools/spec_ab.py C3 12500 2000 default spec_ck=0x790011 2>&1 | tee $O/ab_c3s.txt || exit 1
echo ALL_OK
