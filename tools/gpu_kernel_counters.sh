# Limiter evidence for the kernels below 0.72 of HBM peak: address translation
# (UTCL1), TA / TD busy, L2 -> fabric stalls, against the C2 transpose and the
# C4 rowcopy as reference points.  One rocprofv3 --pmc pass per counter group
# (at most 4 TCP_, 2 TA_, 2 TD_, 4 TCC_ counters a pass), each under a KILL timeout.
set -o pipefail
export TMPDIR=/tmp
OPS="c2swap c4swap c3swap c5T c5pack c5v2k"
i=0
for grp in "TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_STALL_MULTI_MISS_sum TCP_UTCL1_STALL_UTCL2_REQ_OUT_OF_CREDITS_sum" \
           "TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_UTCL1_SERIALIZATION_STALL_sum" \
           "TA_BUSY_avr TA_TA_BUSY_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE" \
           "TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_TAG_STALL_sum" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $grp -d gpurun_out/kc_$i -o pmc --output-format csv -- python tools/kernel_counters.py $OPS > gpurun_out/kc_$i.log 2>&1 || { echo PMC_FAIL $i; exit 1; }
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kc_trace -o run --output-format csv -- python tools/kernel_counters.py $OPS > gpurun_out/kc_trace.log 2>&1 || { echo TRACE_FAIL; exit 1; }
echo ALL_OK
