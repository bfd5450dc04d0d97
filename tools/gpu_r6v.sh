# Round 6: the set-up (staging, validation, cuts) at priority 3 above every TOP
# walk (TOP walks 2,1,0,0 by quarter: LC_SPEC_CUT_PRIO=1 LC_SPEC_PRIO_TOP=2)
# against the default (set-up 0, TOP walks 3,2,1,0).  The stamps showed the
# 4th block on each CU starved through its set-up by the other blocks'
# first-quarter walks and ending last.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6v; mkdir -p $O
L=$PWD/jepsen-etcd-demo_amd/lincheck
for c in C2 C5; do for sd in "" 11 15; do
  SEED=$sd timeout -k 10 200 python -u tools/spec_ab.py $c 1000 1000 default > $O/def_${c}_$sd.txt 2>&1 || { tail -5 $O/def_${c}_$sd.txt; exit 1; }
  SEED=$sd LINCHECK_LIB_OVERRIDE=$L/liblincheck_cp2.so timeout -k 10 200 python -u tools/spec_ab.py $c 1000 1000 default > $O/cp2_${c}_$sd.txt 2>&1 || { tail -5 $O/cp2_${c}_$sd.txt; exit 1; }
  echo "$c seed ${sd:-default}: default $(grep -o 'median [0-9.]*' $O/def_${c}_$sd.txt) / set-up 3, TOP 2,1,0,0 $(grep -o 'median [0-9.]*' $O/cp2_${c}_$sd.txt)"
done; done
export LINCHECK_LIB_OVERRIDE=$L/liblincheck_cp2st.so
SPEC_CFG=C2 timeout -k 10 120 python -u tools/spec_stamps.py 1000 8 0 $O/st_c2.npz > $O/st_c2.txt 2>&1 || { tail $O/st_c2.txt; exit 1; }
SPEC_CFG=C5 timeout -k 10 120 python -u tools/spec_stamps.py 1000 8 0 $O/st_c5.npz > $O/st_c5.txt 2>&1 || { tail $O/st_c5.txt; exit 1; }
