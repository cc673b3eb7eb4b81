# Round 6, call b: the unit-axis GPU tests, the counter list of the box, and
# the C5 .T stride study (tools/c5t_stride_probe.py) with three --pmc passes.
set -o pipefail
export TMPDIR=/tmp
T=${TAG:-r06b}
mkdir -p gpurun_out
timeout -k 10 120 rocprofv3 -L > gpurun_out/${T}_counters.txt 2>&1 || echo "LIST_FAIL (continuing)"
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_golden_api.py tests/test_fuzz_oracle.py > gpurun_out/${T}_gpu_tests.log 2>&1 || { echo TESTS_FAIL; tail -30 gpurun_out/${T}_gpu_tests.log; exit 1; }
tail -2 gpurun_out/${T}_gpu_tests.log
timeout -k 10 300 python -u tools/c5t_stride_probe.py --check --rounds 3 --reps 3 > gpurun_out/${T}_c5t_stride.log 2>&1 || { echo PROBE_FAIL; tail -20 gpurun_out/${T}_c5t_stride.log; exit 1; }
cat gpurun_out/${T}_c5t_stride.log
V=dense,s+256B,s+4KiB,s+2MiB,d+4KiB,sd+4KiB
i=0
for grp in "TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_TAG_STALL_sum" \
           "TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum" \
           "TCC_EA0_WRREQ_STALL_sum TCC_EA0_RDREQ_sum TCP_TCC_WRITE_REQ_LATENCY_sum TCP_TCC_WRITE_REQ_sum"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $grp --kernel-trace -d gpurun_out/${T}_pmc_$i -o pmc --output-format csv -- python tools/c5t_stride_probe.py --rounds 1 --reps 3 --variants $V > gpurun_out/${T}_pmc_$i.log 2>&1 || { echo PMC_FAIL $i; tail -5 gpurun_out/${T}_pmc_$i.log; exit 1; }
done
python tools/c5t_pmc_table.py --variants $V --reps 3 gpurun_out/${T}_pmc_1 gpurun_out/${T}_pmc_2 gpurun_out/${T}_pmc_3 > gpurun_out/${T}_c5t_pmc_table.md && cat gpurun_out/${T}_c5t_pmc_table.md
echo ALL_OK
