# Round 2: the fused 512-B f64 transpose as product default (lib_f512 = the
# tree's build) and XCD-contiguous transpose tiles (BM_TR_XCD), A/B twice
# against the previous build, then the permutation tests of both.
set -o pipefail
export TMPDIR=/tmp
L=tools/ab_libs
T=r02q
for rep in 1 2; do
timeout -k 10 600 python tools/ab_bench.py $L/lib_base.so $L/lib_f512.so $L/lib_trxcd.so --ops c5_T,c5_perm,c2_swap,c3_T,u16_T --rounds 5 > gpurun_out/ab_${T}_$rep.log 2>&1 || { echo AB_FAIL; tail -20 gpurun_out/ab_${T}_$rep.log; exit 1; }
grep -v amdgpu.ids gpurun_out/ab_${T}_$rep.log
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_fuzz_medium.py "tests/test_gpu_large.py::test_transpose_full_size" -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/tests_${T}_product.log 2>&1 || { echo TESTS_FAIL product; tail -30 gpurun_out/tests_${T}_product.log; exit 1; }
echo product; tail -1 gpurun_out/tests_${T}_product.log
BOLT_AMD_LIB=$L/lib_trxcd.so timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_fuzz_medium.py "tests/test_gpu_large.py::test_transpose_full_size" -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/tests_${T}_trxcd.log 2>&1 || { echo TESTS_FAIL trxcd; tail -30 gpurun_out/tests_${T}_trxcd.log; exit 1; }
echo trxcd; tail -1 gpurun_out/tests_${T}_trxcd.log
echo ALL_OK
