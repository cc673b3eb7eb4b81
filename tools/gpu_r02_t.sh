# Round 2: C5 .T with the source-contiguous 512-B rows fused with their source
# continuation (BM_T8_FUSEA; 1-2 KiB read segments), four tile shapes, A/B
# twice, then each variant's permutation tests (incl. the new Diag16 shapes).
set -o pipefail
export TMPDIR=/tmp
L=tools/ab_libs
T=r02t
for rep in 1 2; do
timeout -k 10 600 python tools/ab_bench.py $L/lib_base.so $L/lib_fa128x64.so $L/lib_fa128x32.so $L/lib_fa256x32.so $L/lib_fa64x64.so --ops c5_T,c5_perm,c3_T --rounds 5 > gpurun_out/ab_${T}_$rep.log 2>&1 || { echo AB_FAIL; tail -20 gpurun_out/ab_${T}_$rep.log; exit 1; }
grep -v amdgpu.ids gpurun_out/ab_${T}_$rep.log
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/tests_${T}_product.log 2>&1 || { echo TESTS_FAIL product; tail -30 gpurun_out/tests_${T}_product.log; exit 1; }
echo product; tail -1 gpurun_out/tests_${T}_product.log
for v in fa128x64 fa128x32 fa256x32 fa64x64; do
BOLT_AMD_LIB=$L/lib_$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_fuzz_medium.py "tests/test_gpu_large.py::test_transpose_full_size" -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/tests_${T}_$v.log 2>&1 || { echo TESTS_FAIL $v; tail -30 gpurun_out/tests_${T}_$v.log; exit 1; }
echo $v; tail -1 gpurun_out/tests_${T}_$v.log
done
echo ALL_OK
