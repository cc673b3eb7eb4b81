# Rows-kernel XCD run length (BM_RED_XCD_G variant builds in tools/ab_libs)
# on the C2 step, dense and padded rows, under rocprofv3 --kernel-trace --stats.
set -o pipefail
T=${T:-r05w}
export TMPDIR=/tmp
for lib in default xcdg16 xcdg128 xcdg1024; do
  L=$PWD/bolt_amd/libbolt_mi355x.so
  [ $lib != default ] && L=$PWD/tools/ab_libs/$lib.so
  for p in 0 1; do
    BOLT_AMD_LIB=$L BOLT_AMD_ROW_PITCH=$p timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_${lib}_p$p -o run -- \
        python tools/host_ab.py . 3 20 > gpurun_out/${T}_${lib}_p$p.log 2>&1 || exit 1
  done
done
