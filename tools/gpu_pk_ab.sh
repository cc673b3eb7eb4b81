# uint16 packed transpose with 128x512 tiles (128 KiB LDS, 512/1024 threads): parity, then A/B.
set -o pipefail
export TMPDIR=/tmp
BOLT_AMD_LIB=$PWD/tools/ab_pk1024.so timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_fuzz_medium.py -m gpu -q -x \
  -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pk_tests.log 2>&1 || { echo TEST_FAIL; exit 1; }
timeout -k 10 600 python tools/ab_bench.py tools/ab_base.so tools/ab_pk1024.so tools/ab_pk512.so \
  --ops u16_T,u16_2d --rounds 5 > gpurun_out/ab_pk3.log 2>&1 || { echo AB_FAIL; exit 1; }
echo ALL_OK
