# Round 2: rows-kernel var/std with sums around the lane-0 Welford mean;
# full-size bitwise parity at every BASELINE config (test_gpu_large);
# default bench (C2 + 64 GiB target sub-record with PMC traffic) + rocprof.
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_numerics.py tests/test_golden_api.py tests/test_gpu_kernels.py tests/test_gpu_fuzz_medium.py -m gpu -q --maxfail=30 -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_r02d.log 2>&1 || { echo TESTS_FAIL; tail -30 gpurun_out/gpu_tests_r02d.log; exit 1; }
tail -2 gpurun_out/gpu_tests_r02d.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_large.py -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/gpu_large_r02d.log 2>&1 || { echo LARGE_FAIL; tail -40 gpurun_out/gpu_large_r02d.log; exit 1; }
grep -E "PASSED|FAILED|passed|failed" gpurun_out/gpu_large_r02d.log | tail -20
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r02d_c2 -o run --output-format csv -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-pmc --no-target64 > gpurun_out/prof_r02d_c2.log 2>&1 || { echo PROF_FAIL; exit 1; }
timeout -k 10 900 python bench.py > gpurun_out/bench_r02d_c2.json 2> gpurun_out/bench_r02d_c2.err || { echo BENCH_FAIL; tail gpurun_out/bench_r02d_c2.err; exit 1; }
cat gpurun_out/bench_r02d_c2.json
echo ALL_OK
