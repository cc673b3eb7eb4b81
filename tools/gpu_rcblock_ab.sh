# Blocked rowcopy traversal (BM_RC_BLOCK) for far-striding rows: parity, then A/B.
set -o pipefail
export TMPDIR=/tmp
BOLT_AMD_LIB=$PWD/tools/ab_blk64.so timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_fuzz_medium.py tests/test_chunk_paths.py -m gpu -q -x \
  -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/rcblock_tests.log 2>&1 || { echo TEST_FAIL; exit 1; }
timeout -k 10 900 python tools/ab_bench.py tools/ab_base.so tools/ab_blk64.so tools/ab_blk256.so tools/ab_blk1024.so \
  --ops c3_full,t64_swap,c4_full,c3_swap --rounds 3 --reps 3 > gpurun_out/ab_rcblock.log 2>&1 || { echo AB_FAIL; exit 1; }
echo ALL_OK
