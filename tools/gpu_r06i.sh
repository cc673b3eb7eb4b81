# Round 6, call i: why column reductions (64 GiB target over axis 0: 0.80-0.85)
# read slower than row reductions (0.87): translation, L1 and DRAM counters
# of the column kernel against the rows kernel on the same bytes.
set -o pipefail
export TMPDIR=/tmp
T=${TAG:-r06i}
mkdir -p gpurun_out
L=bolt_amd/libbolt_mi355x.so
OPS=t64_mean_cols,t64_std_cols,c2_mean_cols,c2_mean_prow,c2_std_prow
timeout -k 10 300 python -u tools/ab_bench.py $L --ops $OPS --rounds 3 --reps 5 > gpurun_out/${T}_times.log 2>&1 || { echo AB_FAIL; tail gpurun_out/${T}_times.log; exit 1; }
cat gpurun_out/${T}_times.log
i=0
for grp in "TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum" \
           "TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_TAG_STALL_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $grp --kernel-trace -d gpurun_out/${T}_pmc_$i -o pmc --output-format csv -- python tools/ab_bench.py $L --ops $OPS --rounds 1 --reps 1 > gpurun_out/${T}_pmc_$i.log 2>&1 || { echo PMC_FAIL $i; tail -5 gpurun_out/${T}_pmc_$i.log; exit 1; }
done
python tools/ab_pmc_table.py --ops t64_mean_cols,t64_std_cols,c2_mean_cols --libs lib --kernel k_red_cols gpurun_out/${T}_pmc_1 gpurun_out/${T}_pmc_2 > gpurun_out/${T}_table.md
python tools/ab_pmc_table.py --ops c2_mean_prow,c2_std_prow --libs lib --kernel k_red_rows gpurun_out/${T}_pmc_1 gpurun_out/${T}_pmc_2 >> gpurun_out/${T}_table.md
cat gpurun_out/${T}_table.md
echo ALL_OK
