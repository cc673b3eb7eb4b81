# Zero-copy statistics results: parity, wall-time probe, C2 bench + kernel trace.
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_api.py tests/test_golden_api.py tests/test_abi.py -m gpu -q -x \
  -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/zc_tests.log 2>&1 || { echo TEST_FAIL; exit 1; }
timeout -k 10 300 python tools/zero_copy_probe.py > gpurun_out/zc_probe.log 2>&1 || { echo PROBE_FAIL; exit 1; }
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-pmc > gpurun_out/bench_c2_zc.json 2> gpurun_out/bench_c2_zc.err || { echo BENCH_FAIL; exit 1; }
BOLT_AMD_ZERO_COPY=0 timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-pmc > gpurun_out/bench_c2_nozc.json 2> gpurun_out/bench_c2_nozc.err || { echo BENCH_FAIL; exit 1; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_zc -o run --output-format csv -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-pmc > gpurun_out/prof_zc.log 2>&1 || { echo PROF_FAIL; exit 1; }
echo ALL_OK
