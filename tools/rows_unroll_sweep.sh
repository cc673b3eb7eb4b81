# Rows-kernel loads in flight (BM_ROWS_UNROLL variant builds in tools/ab_libs)
# on the C2 step with padded rows, under rocprofv3 --kernel-trace --stats.
set -o pipefail
T=${T:-r05z}
export TMPDIR=/tmp
for lib in default unroll3 unroll4; do
  L=$PWD/bolt_amd/libbolt_mi355x.so
  [ $lib != default ] && L=$PWD/tools/ab_libs/$lib.so
  BOLT_AMD_LIB=$L timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_$lib -o run -- \
      python tools/host_ab.py . 3 20 > gpurun_out/${T}_$lib.log 2>&1 || exit 1
done
