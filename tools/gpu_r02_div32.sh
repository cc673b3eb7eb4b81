# A/B: transpose tile coordinates in 32-bit (new default) vs 64-bit mul-hi
# (tools/ab_libs/div0.so, -DBM_TR_DIV32=0), interleaved in one process.
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python tools/ab_bench.py bolt_amd/libbolt_mi355x.so tools/ab_libs/div0.so --ops c5_T,c5_perm,c2_swap,c3_T,u16_T,u8_T --rounds 5 > gpurun_out/r02_ab_div32.log 2>&1 || { echo AB_FAIL; tail -20 gpurun_out/r02_ab_div32.log; exit 1; }
cat gpurun_out/r02_ab_div32.log
