# Round 2: column reductions (the 64 GiB target's mean / std over axis 0, C4's
# var) -- rows in flight per lane (BM_COLS_UNROLL 2 / 8) and splitting R over
# more blocks (BM_COLS_BLOCKS 4096 / 8192), A/B twice.
set -o pipefail
export TMPDIR=/tmp
L=tools/ab_libs
T=r02r
for rep in 1 2; do
timeout -k 10 600 python tools/ab_bench.py $L/lib_base.so $L/lib_u8.so $L/lib_u2.so $L/lib_b4k.so $L/lib_b8k.so --ops t64f_mean_cols,t64f_std_cols,c4_var_full,c2_mean_cols,c2_std_cols --rounds 5 > gpurun_out/ab_${T}_$rep.log 2>&1 || { echo AB_FAIL; tail -20 gpurun_out/ab_${T}_$rep.log; exit 1; }
grep -v amdgpu.ids gpurun_out/ab_${T}_$rep.log
done
echo ALL_OK
