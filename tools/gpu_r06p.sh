# Round 6, call p: kernel time against the XCD its block 0 lands on
# (tools/xcd_offset_probe.py): the dispatch model checked, then C5 pack / .T /
# v2k repack and the C2 swap with block 0 steered to each XCD.
set -o pipefail
export TMPDIR=/tmp
T=${TAG:-r06p}
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/xcd_offset_probe.py --ops c5_pack,c5_T,c5_v2k,c2_swap --rounds 4 --reps 2 > gpurun_out/${T}_xcd_offset.log 2>&1 || { echo PROBE_FAIL; tail -20 gpurun_out/${T}_xcd_offset.log; exit 1; }
cat gpurun_out/${T}_xcd_offset.log
echo ALL_OK
