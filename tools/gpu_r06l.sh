# Round 6, call l: column kernels' rows in flight per lane (kColsUnroll 4 / 8 /
# 16) on the 64-vector tiles, interleaved, two placements.
set -o pipefail
export TMPDIR=/tmp
T=${TAG:-r06l}
mkdir -p gpurun_out
V="tools/ab_libs/cols_u8.so tools/ab_libs/cols_u4.so tools/ab_libs/cols_u16.so"
timeout -k 10 300 python -u tools/cols_numerics_check.py $V > gpurun_out/${T}_numerics.log 2>&1 || { echo NUM_FAIL; tail gpurun_out/${T}_numerics.log; }
cat gpurun_out/${T}_numerics.log
timeout -k 10 900 python -u tools/ab_bench.py $V --ops t64f_mean_cols,t64f_std_cols,c2_mean_cols,c2_std_cols --rounds 5 --reps 3 --placements 2 > gpurun_out/${T}_ab.log 2>&1 || { echo AB_FAIL; tail gpurun_out/${T}_ab.log; exit 1; }
cat gpurun_out/${T}_ab.log
echo ALL_OK
