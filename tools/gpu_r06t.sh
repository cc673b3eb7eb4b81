# Round 6, call t: k_transpose with the non-temporal hint dropped on its loads
# (t_tld), its stores (t_tst) or both (t_tboth), against the shipped build, on
# C5 .T, the C2 swap and C3 .T, two placements, outputs compared.
set -o pipefail
export TMPDIR=/tmp
T=${TAG:-r06t}
mkdir -p gpurun_out
L="tools/ab_libs/t_base.so tools/ab_libs/t_tld.so tools/ab_libs/t_tst.so tools/ab_libs/t_tboth.so"
timeout -k 10 700 python -u tools/dst_placement_ab.py $L --ops c5_T,c2_swap,c3_T --k 2 --kinds hipmalloc,vmm --rounds 2 --reps 3 --check > gpurun_out/${T}_nt.log 2>&1 || { echo AB_FAIL; tail -20 gpurun_out/${T}_nt.log; exit 1; }
cat gpurun_out/${T}_nt.log
echo ALL_OK
