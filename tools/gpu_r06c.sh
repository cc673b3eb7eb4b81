# Round 6, call c: (1) the rows kernel's pivot taken from its first vector
# load (tools/ab_libs/rows_peel.so) against the shipped build (rows_base.so):
# byte identity, interleaved timing, FETCH / WRITE bytes per launch;
# (2) the C5 pack placement study with write-side and translation counters;
# (3) the C5 pack in three fresh processes.
set -o pipefail
export TMPDIR=/tmp
T=${TAG:-r06c}
mkdir -p gpurun_out
B=tools/ab_libs/rows_base.so
P=tools/ab_libs/rows_peel.so
timeout -k 10 300 python -u tools/rows_peel_check.py $B $P > gpurun_out/${T}_peel_check.log 2>&1 || { echo CHECK_FAIL; tail -20 gpurun_out/${T}_peel_check.log; exit 1; }
tail -1 gpurun_out/${T}_peel_check.log
OPS=c2_mean_prow,c2_std_prow,c2_mean_rows,c2_std_rows,c2q_mean_prow,c2q_std_prow,c2_sum_prow
timeout -k 10 300 python -u tools/ab_bench.py $B $P --ops $OPS --rounds 7 --reps 10 > gpurun_out/${T}_ab_peel.log 2>&1 || { echo AB_FAIL; tail -20 gpurun_out/${T}_ab_peel.log; exit 1; }
cat gpurun_out/${T}_ab_peel.log
OPS2=c2_mean_prow,c2_std_prow,c2_sum_prow,c2_max_prow,c2_mean_rows,c2_std_rows,c2_sum_rows,c2q_mean_prow
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $c --kernel-trace -d gpurun_out/${T}_red_$c -o pmc --output-format csv -- python tools/ab_bench.py $B $P --ops $OPS2 --rounds 1 --reps 1 > gpurun_out/${T}_red_$c.log 2>&1 || { echo PMC_FAIL $c; tail -5 gpurun_out/${T}_red_$c.log; exit 1; }
done
python tools/ab_pmc_table.py --ops $OPS2 --libs base,peel --kernel k_red_rows gpurun_out/${T}_red_FETCH_SIZE gpurun_out/${T}_red_WRITE_SIZE > gpurun_out/${T}_red_traffic.md && cat gpurun_out/${T}_red_traffic.md
K="--matrix 3 --matrix-kinds hipmalloc"
timeout -k 10 300 python -u tools/alloc_kind_probe.py $K --rounds 3 --reps 5 --ops c5_pack > gpurun_out/${T}_pack_matrix.log 2>&1 || { echo MATRIX_FAIL; tail -20 gpurun_out/${T}_pack_matrix.log; exit 1; }
cat gpurun_out/${T}_pack_matrix.log
i=0
for grp in "TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_STALL_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_TAG_STALL_sum" \
           "TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_STALL_UTCL2_REQ_OUT_OF_CREDITS_sum TCP_UTCL1_TRANSLATION_MISS_UNDER_MISS_sum GRBM_UTCL2_BUSY GRBM_GUI_ACTIVE" \
           "TCC_EA0_WRREQ_LEVEL_sum TCC_EA0_RDREQ_LEVEL_sum TCP_TCC_WRITE_REQ_LATENCY_sum TCP_TCC_WRITE_REQ_sum"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $grp --kernel-trace -d gpurun_out/${T}_pack_pmc_$i -o pmc --output-format csv -- python tools/alloc_kind_probe.py $K --rounds 1 --reps 1 --ops c5_pack > gpurun_out/${T}_pack_pmc_$i.log 2>&1 || { echo PACK_PMC_FAIL $i; tail -5 gpurun_out/${T}_pack_pmc_$i.log; break; }
  python tools/placement_pmc_table.py gpurun_out/${T}_pack_pmc_$i --k 3 > gpurun_out/${T}_pack_pmc_table_$i.txt && cat gpurun_out/${T}_pack_pmc_table_$i.txt
done
for i in 1 2 3; do
  timeout -k 10 120 python -u tools/ab_bench.py bolt_amd/libbolt_mi355x.so --ops c5_pack,c5_T --rounds 3 --reps 5 > gpurun_out/${T}_fresh_$i.log 2>&1 || { echo FRESH_FAIL $i; exit 1; }
  cat gpurun_out/${T}_fresh_$i.log
done
echo ALL_OK
