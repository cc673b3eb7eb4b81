# Round 6, call j: column-reduction variants (tools/ab_libs/cols_*.so) --
# narrower column tiles (128 / 64 vectors: more row phases) and 32 B per lane
# for 4- / 8-byte elements -- against the shipped build, interleaved.
set -o pipefail
export TMPDIR=/tmp
T=${TAG:-r06j}
mkdir -p gpurun_out
V="tools/ab_libs/cols_base.so tools/ab_libs/cols_t128.so tools/ab_libs/cols_t64.so tools/ab_libs/cols_v8.so"
timeout -k 10 300 python -u tools/cols_numerics_check.py $V > gpurun_out/${T}_numerics.log 2>&1 || { echo NUM_FAIL; tail gpurun_out/${T}_numerics.log; }
cat gpurun_out/${T}_numerics.log
timeout -k 10 600 python -u tools/ab_bench.py $V --ops t64f_mean_cols,t64f_std_cols,c2_mean_cols,c2_std_cols,c4_var_cols,c4_var_full --rounds 5 --reps 3 > gpurun_out/${T}_ab.log 2>&1 || { echo AB_FAIL; tail gpurun_out/${T}_ab.log; exit 1; }
cat gpurun_out/${T}_ab.log
echo ALL_OK
