# Wave-per-row rowcopy: parity with the variant library, then A/B.
set -o pipefail
export TMPDIR=/tmp
BOLT_AMD_LIB=$PWD/tools/ab_rw512.so timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_fuzz_medium.py tests/test_chunk_paths.py -m gpu -q -x \
  -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/rcw_tests.log 2>&1 || { echo TEST_FAIL; exit 1; }
timeout -k 10 600 python tools/ab_bench.py tools/ab_rw0.so tools/ab_rw512.so tools/ab_rw2048.so tools/ab_rw512u2.so \
  --ops c5_k2v,c4_swap,c4_full,c2_copy > gpurun_out/ab_rcw.log 2>&1 || { echo AB_FAIL; exit 1; }
echo ALL_OK
