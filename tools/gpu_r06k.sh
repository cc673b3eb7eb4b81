# Round 6, call k: the narrower column tiles (cols_t64.so, kColsTcv 64) against
# the shipped build, reversed order, two buffer placements per op.
set -o pipefail
export TMPDIR=/tmp
T=${TAG:-r06k}
mkdir -p gpurun_out
timeout -k 10 900 python -u tools/ab_bench.py tools/ab_libs/cols_t64.so tools/ab_libs/cols_t128.so tools/ab_libs/cols_base.so --ops t64f_mean_cols,t64f_std_cols,t64_mean_cols,t64_std_cols,c2_mean_cols,c4_var_full --rounds 5 --reps 3 --placements 2 > gpurun_out/${T}_ab.log 2>&1 || { echo AB_FAIL; tail gpurun_out/${T}_ab.log; exit 1; }
cat gpurun_out/${T}_ab.log
echo ALL_OK
