# Placement study: the source x destination matrix of
# C5 .T and C5 pack over four allocation kinds, timed, then the same matrix
# (1 call per pair after 2 warm-ups) under two rocprofv3 --pmc passes with the
# kernel trace, to correlate per-buffer speed with translation / L2 counters.
set -o pipefail
export TMPDIR=/tmp
T=${TAG:-r03h}
K="--matrix 4 --matrix-kinds hipmalloc,contiguous,vmm,hipmalloc"
timeout -k 10 300 python -u tools/alloc_kind_probe.py $K --rounds 3 --reps 5 --ops c5_T,c5_pack > gpurun_out/${T}_matrix.log 2>&1 || { echo MATRIX_FAIL; tail -20 gpurun_out/${T}_matrix.log; exit 1; }
cat gpurun_out/${T}_matrix.log
i=0
for grp in "TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_STALL_MULTI_MISS_sum TCP_UTCL1_STALL_UTCL2_REQ_OUT_OF_CREDITS_sum" \
           "TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_TAG_STALL_sum"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $grp --kernel-trace -d gpurun_out/${T}_pmc_$i -o pmc --output-format csv -- python tools/alloc_kind_probe.py $K --rounds 1 --reps 1 --ops c5_T,c5_pack > gpurun_out/${T}_pmc_$i.log 2>&1 || { echo PMC_FAIL $i; tail -5 gpurun_out/${T}_pmc_$i.log; exit 1; }
done
echo ALL_OK
