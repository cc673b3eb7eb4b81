# packed transpose tile / thread-count variants: parity, then A/B.
set -o pipefail
export TMPDIR=/tmp
for v in base u8d u16g; do
BOLT_AMD_LIB=$PWD/tools/ab_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_fuzz_medium.py -m gpu -q -x \
  -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pk8_tests_$v.log 2>&1 || { echo TEST_FAIL $v; exit 1; }
done
timeout -k 10 600 python tools/ab_bench.py tools/ab_base.so tools/ab_u8d.so tools/ab_u8e.so tools/ab_u8f.so tools/ab_u16g.so \
  --ops u8_T,u16_T,u16_2d --rounds 5 > gpurun_out/ab_pk5.log 2>&1 || { echo AB_FAIL; exit 1; }
echo ALL_OK
