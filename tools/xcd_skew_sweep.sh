# Rows kernel: each XCD walks its eighth of the rows from a rotated start
# (BM_RED_XCD_SKEW variant builds), C2 step, rocprofv3; alternating builds.
#   LIBS="default skew37" PITCH="1 0" ROUNDS=2 bash tools/xcd_skew_sweep.sh
set -o pipefail
T=${T:-r05zc}
export TMPDIR=/tmp
for r in $(seq 1 ${ROUNDS:-1}); do
for lib in ${LIBS:-default skew37 skew613}; do
  L=$PWD/bolt_amd/libbolt_mi355x.so
  [ $lib != default ] && L=$PWD/tools/ab_libs/$lib.so
  for p in ${PITCH:-1 0}; do
    BOLT_AMD_LIB=$L BOLT_AMD_ROW_PITCH=$p timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_${lib}_p${p}_$r -o run -- \
        python tools/host_ab.py . ${REPS:-3} ${STEPS:-20} > gpurun_out/${T}_${lib}_p${p}_$r.log 2>&1 || exit 1
  done
done
done
