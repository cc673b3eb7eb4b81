# Loads-first runs transpose (BM_RUNS_LF, up to 128-B runs) and unpredicated
# interior transpose tiles (BM_TP_INTERIOR): parity with the variants, then A/B.
set -o pipefail
export TMPDIR=/tmp
for v in rlf128tb32 tpi; do
  BOLT_AMD_LIB=$PWD/tools/ab_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_fuzz_medium.py -m gpu -q -x \
    -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/runs_tests_$v.log 2>&1 || { echo TEST_FAIL $v; exit 1; }
done
timeout -k 10 900 python tools/ab_bench.py tools/ab_base.so tools/ab_rlf.so tools/ab_rlf128.so tools/ab_rlf128tb32.so tools/ab_tpi.so \
  --ops runs32,runs64,runs128,c3_swap,c2_swap,c5_T,c5_perm,c3_T --rounds 5 > gpurun_out/ab_runs.log 2>&1 || { echo AB_FAIL; exit 1; }
echo ALL_OK
