# Write-side limiter counters of the record scatter (k_recmap_scatter): C5
# keys_to_values((2,)) at 0.69-0.71 of HBM against C5 unchunk (same kernel,
# 0.81) and the C4 rowcopy.  One rocprofv3 --pmc pass per group (<= 4 TCC_,
# 4 TCP_, 2 GRBM_ counters), each under a KILL timeout; then a kernel trace.
set -o pipefail
export TMPDIR=/tmp
T=${TAG:-r04a}
OPS="c5k2v c5unchunk c4swap"
i=0
for grp in "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCP_TCC_WRITE_REQ_sum TCP_TCC_WRITE_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum TCP_WRITE_TAGCONFLICT_STALL_CYCLES_sum" \
           "TCC_EA0_WRREQ_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_LEVEL_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum GRBM_GUI_ACTIVE" \
           "TCC_EA0_WR_UNCACHED_32B_sum TCC_TAG_STALL_sum TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_RDREQ_sum" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $grp -d gpurun_out/${T}_sc_$i -o pmc --output-format csv -- python tools/scatter_counters.py $OPS > gpurun_out/${T}_sc_$i.log 2>&1 || { echo PMC_FAIL $i; tail -5 gpurun_out/${T}_sc_$i.log; exit 1; }
  echo pass $i done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_sc_trace -o run --output-format csv -- python tools/scatter_counters.py $OPS > gpurun_out/${T}_sc_trace.log 2>&1 || { echo TRACE_FAIL; exit 1; }
echo ALL_OK
