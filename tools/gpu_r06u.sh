# Round 6, call u: the C5 pack through the direct record map (no LDS
# staging: every destination element read from the source through the map)
# against the LDS-staged kernel, three placements, outputs compared.
set -o pipefail
export TMPDIR=/tmp
T=${TAG:-r06u}
mkdir -p gpurun_out
timeout -k 10 500 python -u tools/dst_placement_ab.py tools/ab_libs/p_base.so tools/ab_libs/p_direct.so --ops c5_pack,c5_pack_copy --k 3 --rounds 2 --reps 3 --check > gpurun_out/${T}_direct.log 2>&1 || { echo AB_FAIL; tail -20 gpurun_out/${T}_direct.log; exit 1; }
cat gpurun_out/${T}_direct.log
echo ALL_OK
