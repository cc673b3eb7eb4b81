# A/B: transpose balanced b-tiles (BM_TR_BAL=1, tools/ab_libs/bal1.so) vs the
# in-tree default, C2 becomes 8 x 252 rows; outputs checked
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 700 python tools/ab_bench.py bolt_amd/libbolt_mi355x.so tools/ab_libs/bal1.so --ops c2_swap,c5_T,c5_perm,c3_T,u16_T,u8_T,u16_2d --rounds 7 --check > gpurun_out/r02_ab_bal.log 2>&1 || { echo AB_FAIL; tail -20 gpurun_out/r02_ab_bal.log; exit 1; }
cat gpurun_out/r02_ab_bal.log
