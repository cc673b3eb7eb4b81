# Round 2: reduction numerics follow-up (table-driven Welford weights) --
# the statistics / reduce / comm GPU tests, smoke, C2 bench + rocprofv3 summary.
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_numerics.py tests/test_gpu_comm.py tests/test_golden_api.py tests/test_gpu_kernels.py -m gpu -q --maxfail=30 -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_r02c.log 2>&1 || { echo TESTS_FAIL; tail -30 gpurun_out/gpu_tests_r02c.log; exit 1; }
tail -2 gpurun_out/gpu_tests_r02c.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r02c_c2 -o run --output-format csv -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-pmc > gpurun_out/prof_r02c_c2.log 2>&1 || { echo PROF_FAIL; exit 1; }
timeout -k 10 600 python bench.py --no-pmc --no-cpu-baseline > gpurun_out/bench_r02c_c2.json 2> gpurun_out/bench_r02c_c2.err || { echo BENCH_FAIL; exit 1; }
cat gpurun_out/bench_r02c_c2.json
echo ALL_OK
