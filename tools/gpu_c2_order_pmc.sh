# Counter study of the C2 transpose's two placement classes:
# timed classification, then two rocprofv3 --pmc passes of the same probe.
#   make -C bolt_amd/csrc OUT=$PWD/tools/ab_libs/inorder.so BUILD=/tmp/bio EXTRA=-DBM_TR_AROT=0
#   make -C bolt_amd/csrc OUT=$PWD/tools/ab_libs/stagger.so BUILD=/tmp/bst EXTRA=-DBM_TR_AROT_FORCE=1
#   TAG=r03zj bash tools/gpu_c2_order_pmc.sh
set -o pipefail
export TMPDIR=/tmp
T=${TAG:-r03zj}
L="tools/ab_libs/inorder.so tools/ab_libs/stagger.so"
timeout -k 10 300 python -u tools/c2_order_probe.py $L --k 6 --reps 3 > gpurun_out/${T}_classes.log 2>&1 || { echo PROBE_FAIL; tail -20 gpurun_out/${T}_classes.log; exit 1; }
cat gpurun_out/${T}_classes.log
i=0
for grp in "TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_TAG_STALL_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum" \
           "TCC_EA0_WRREQ_STALL_sum TCC_EA0_RDREQ_sum TCP_TCC_WRITE_REQ_LATENCY_sum TCP_TCC_WRITE_REQ_sum"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $grp --kernel-trace -d gpurun_out/${T}_pmc_$i -o pmc --output-format csv -- python tools/c2_order_probe.py $L --k 6 --reps 3 > gpurun_out/${T}_pmc_$i.log 2>&1 || { echo PMC_FAIL $i; tail -5 gpurun_out/${T}_pmc_$i.log; exit 1; }
  python tools/c2_order_pmc_table.py gpurun_out/${T}_pmc_$i --k 6 --reps 3 > gpurun_out/${T}_pmc_table_$i.txt && cat gpurun_out/${T}_pmc_table_$i.txt
done
echo ALL_OK
