# Round 6: segments per key on C2 / C5 with the spill-free builds, and the
# drop-in call's host split (pack phases, shaping) on the box.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6c
mkdir -p $O
timeout -k 10 200 python -u tools/spec_ab.py C2 1000 1000 default spec_segs=4 spec_segs=8 > $O/ab_c2.txt 2>&1 || { tail -5 $O/ab_c2.txt; exit 1; }
cat $O/ab_c2.txt
timeout -k 10 200 python -u tools/spec_ab.py C5 1000 1000 default spec_segs=4 spec_segs=8 > $O/ab_c5.txt 2>&1 || { tail -5 $O/ab_c5.txt; exit 1; }
cat $O/ab_c5.txt
LC_TIMING=1 timeout -k 10 200 python -u tools/jepsen_profile.py > $O/jepsen_profile.txt 2> $O/jepsen_timing.txt || { tail -5 $O/jepsen_profile.txt; exit 1; }
head -14 $O/jepsen_profile.txt
tail -12 $O/jepsen_timing.txt
