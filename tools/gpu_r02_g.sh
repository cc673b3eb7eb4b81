# Round 2: page-locality batch order for transposes (+ rowcopy diagonal walk,
# XCD-contiguous reduction rows) A/B in one process, and the combined build's
# correctness (every 4-d permutation kernel test, medium fuzz, full-size parity).
set -o pipefail
export TMPDIR=/tmp
L=tools/ab_libs
timeout -k 10 700 python tools/ab_bench.py $L/lib_base.so $L/lib_page.so $L/lib_pagerc.so --ops c5_T,c5_perm,c3_T,c2_swap,c4_full,u16_T,u8_T,c3_full,t64_swap,c2_mean_rows,c2_std_rows,c5_k2v --rounds 5 > gpurun_out/ab_page_r02g.log 2>&1 || { echo AB_FAIL; tail -20 gpurun_out/ab_page_r02g.log; exit 1; }
grep -v amdgpu.ids gpurun_out/ab_page_r02g.log
BOLT_AMD_LIB=$L/lib_pagerc.so timeout -k 10 900 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_fuzz_medium.py tests/test_golden_api.py tests/test_gpu_large.py -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pagerc_tests_r02g.log 2>&1 || { echo TESTS_FAIL; tail -30 gpurun_out/pagerc_tests_r02g.log; exit 1; }
tail -2 gpurun_out/pagerc_tests_r02g.log
echo ALL_OK
