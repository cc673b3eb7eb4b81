# Round 6, call r: C5 pack / .T against the copy ceiling of the same
# destination, over hipMalloc / contiguous / VMM placements.
set -o pipefail
export TMPDIR=/tmp
T=${TAG:-r06r}
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/dst_placement_ab.py bolt_amd/libbolt_mi355x.so --ops c5_pack,c5_pack_copy,c5_T,c5_T_copy,c5_v2k --k 3 --rounds 2 --reps 2 > gpurun_out/${T}_dst.log 2>&1 || { echo DST_FAIL; tail -20 gpurun_out/${T}_dst.log; exit 1; }
cat gpurun_out/${T}_dst.log
echo ALL_OK
