# Round 2: 16x16 diagonal-tile rowcopy (BM_RC_DIAG) A/B on the 128-B-row
# swaps, twice in one session, and its correctness on the permutation tests.
set -o pipefail
export TMPDIR=/tmp
L=tools/ab_libs
for rep in 1 2; do
timeout -k 10 600 python tools/ab_bench.py $L/lib_base.so $L/lib_diag.so --ops c3_full,t64_swap,c3_swap,c4_full,c5_k2v --rounds 5 > gpurun_out/ab_diag_r02m_$rep.log 2>&1 || { echo AB_FAIL; tail -20 gpurun_out/ab_diag_r02m_$rep.log; exit 1; }
grep -v amdgpu.ids gpurun_out/ab_diag_r02m_$rep.log
done
BOLT_AMD_LIB=$L/lib_diag.so timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_fuzz_medium.py "tests/test_gpu_large.py::test_swap_full_size" "tests/test_gpu_large.py::test_target64_swap_full_size" -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/diag_tests_r02m.log 2>&1 || { echo TESTS_FAIL; tail -30 gpurun_out/diag_tests_r02m.log; exit 1; }
tail -2 gpurun_out/diag_tests_r02m.log
echo ALL_OK
