# Round 6, call e: the rows kernel with a wave-uniform main loop
# (tools/ab_libs/rows_wave.so) against the shipped build (rows_base.so):
# numerics against long double, interleaved timing, read bytes per launch.
set -o pipefail
export TMPDIR=/tmp
T=${TAG:-r06e}
mkdir -p gpurun_out
B=tools/ab_libs/rows_base.so
W=tools/ab_libs/rows_wave.so
timeout -k 10 300 python -u tools/rows_numerics_check.py $B $W > gpurun_out/${T}_numerics.log 2>&1 || { echo NUM_FAIL; cat gpurun_out/${T}_numerics.log | tail; exit 1; }
cat gpurun_out/${T}_numerics.log
OPS=c2_mean_prow,c2_std_prow,c2_mean_rows,c2_std_rows,c2q_mean_prow,c2q_std_prow,c2_sum_prow,c2_max_prow
timeout -k 10 300 python -u tools/ab_bench.py $B $W --ops $OPS --rounds 7 --reps 10 > gpurun_out/${T}_ab.log 2>&1 || { echo AB_FAIL; tail -20 gpurun_out/${T}_ab.log; exit 1; }
cat gpurun_out/${T}_ab.log
timeout -k 10 300 python -u tools/ab_bench.py $W $B --ops $OPS --rounds 7 --reps 10 > gpurun_out/${T}_ab_rev.log 2>&1 || { echo AB_FAIL; exit 1; }
cat gpurun_out/${T}_ab_rev.log
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/${T}_fetch -o pmc --output-format csv -- python tools/ab_bench.py $B $W --ops $OPS --rounds 1 --reps 1 > gpurun_out/${T}_fetch.log 2>&1 || { echo PMC_FAIL; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_64B_sum --kernel-trace -d gpurun_out/${T}_rq -o pmc --output-format csv -- python tools/ab_bench.py $B $W --ops $OPS --rounds 1 --reps 1 > gpurun_out/${T}_rq.log 2>&1 || { echo PMC_FAIL; exit 1; }
python tools/ab_pmc_table.py --ops $OPS --libs base,wave --kernel k_red_rows gpurun_out/${T}_fetch gpurun_out/${T}_rq > gpurun_out/${T}_traffic.md && cat gpurun_out/${T}_traffic.md
echo ALL_OK
