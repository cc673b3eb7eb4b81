# uint16 packed-transpose tile sweep (BM_PK16_TA x TB, NT threads), outputs checked against torch
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 800 python tools/ab_bench.py bolt_amd/libbolt_mi355x.so tools/ab_libs/pk16_A.so tools/ab_libs/pk16_B.so tools/ab_libs/pk16_C.so tools/ab_libs/pk16_D.so tools/ab_libs/pk16_E.so --ops u16_T,u16_2d --rounds 5 --check > gpurun_out/r02_ab_pk16.log 2>&1 || { echo AB_FAIL; tail -20 gpurun_out/r02_ab_pk16.log; exit 1; }
cat gpurun_out/r02_ab_pk16.log
