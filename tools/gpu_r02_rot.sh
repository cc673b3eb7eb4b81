# A/B: transpose tiles rotated per a-row (BM_TR_ROT=1, tools/ab_libs/rot1.so) vs the
# in-tree default, so C2's partial b-tile is spread over all 8 XCDs; outputs checked
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 700 python tools/ab_bench.py bolt_amd/libbolt_mi355x.so tools/ab_libs/rot1.so --ops c2_swap,c5_T,c5_perm,c3_T,u16_T,u8_T,u16_2d --rounds 7 --check > gpurun_out/r02_ab_rot.log 2>&1 || { echo AB_FAIL; tail -20 gpurun_out/r02_ab_rot.log; exit 1; }
cat gpurun_out/r02_ab_rot.log
