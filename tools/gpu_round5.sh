set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "beyond or reduce" -m gpu -q -x -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/tests5.log 2>&1 || { echo TESTS_FAIL; exit 1; }
timeout -k 10 600 python tools/ab_bench.py tools/ab_A.so tools/ab_B.so tools/ab_C.so --ops c3_swap,c4_swap,runs128,c2_copy,c5_T > gpurun_out/ab_rc.log 2>&1 || { echo AB_FAIL; exit 1; }
timeout -k 10 600 python bench.py --config target64 --steps 5 --warmup 1 --no-cpu-baseline --no-pmc > gpurun_out/bench_target64.json 2> gpurun_out/bench_target64.err || { echo BENCH_FAIL; exit 1; }
echo ALL_OK
