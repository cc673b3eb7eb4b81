# Round 6, call q: the slow state (C5 pack 4.0 ms instead of 3.2-3.4, C2 swap
# 0.74 instead of 0.67): shader clock from GRBM_COUNT / GRBM_GUI_ACTIVE per
# launch, with and without idle gaps between launches.
set -o pipefail
export TMPDIR=/tmp
T=${TAG:-r06q}
mkdir -p gpurun_out
(rocm-smi --showclocks > gpurun_out/${T}_clocks_before.txt 2>&1 || true)
timeout -k 10 120 python -u tools/ab_bench.py bolt_amd/libbolt_mi355x.so --ops c5_pack,c2_swap,c5_T --rounds 3 --reps 5 > gpurun_out/${T}_ab.log 2>&1 || { echo AB_FAIL; tail -20 gpurun_out/${T}_ab.log; exit 1; }
cat gpurun_out/${T}_ab.log
timeout -k 10 200 python -u tools/xcd_offset_probe.py --ops c5_pack,c2_swap --rounds 2 --reps 2 > gpurun_out/${T}_xcd.log 2>&1 || { echo PROBE_FAIL; tail -20 gpurun_out/${T}_xcd.log; exit 1; }
grep -v steer gpurun_out/${T}_xcd.log
timeout -s KILL 120 rocprofv3 --pmc GRBM_COUNT GRBM_GUI_ACTIVE --kernel-trace -d gpurun_out/${T}_pmc_ab -o pmc --output-format csv -- python tools/ab_bench.py bolt_amd/libbolt_mi355x.so --ops c5_pack,c2_swap --rounds 1 --reps 3 > gpurun_out/${T}_pmc_ab.log 2>&1 || { echo PMC_AB_FAIL; tail -5 gpurun_out/${T}_pmc_ab.log; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc GRBM_COUNT GRBM_GUI_ACTIVE --kernel-trace -d gpurun_out/${T}_pmc_xcd -o pmc --output-format csv -- python tools/xcd_offset_probe.py --ops c5_pack,c2_swap --rounds 1 --reps 1 > gpurun_out/${T}_pmc_xcd.log 2>&1 || { echo PMC_XCD_FAIL; tail -5 gpurun_out/${T}_pmc_xcd.log; exit 1; }
python tools/clock_pmc_table.py gpurun_out/${T}_pmc_ab gpurun_out/${T}_pmc_xcd
(rocm-smi --showclocks > gpurun_out/${T}_clocks_after.txt 2>&1 || true)
echo ALL_OK
