set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_api.py tests/test_golden_api.py -m gpu -q -x -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/tests6.log 2>&1 || { echo TESTS_FAIL; exit 1; }
timeout -k 10 600 python tools/ab_bench.py tools/ab_nopk.so tools/ab_pk.so --ops u16_T,u8_T,u16_2d,c2_swap > gpurun_out/ab_pk.log 2>&1 || { echo AB_FAIL; exit 1; }
echo ALL_OK
