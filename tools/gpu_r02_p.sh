# Round 2: f64 transposes with 512-B destination rows (C5 .T / transpose(2,0,4,1,3)):
# fuse the destination-contiguous axis with its continuation and use longer
# write segments (BM_T8_FUSE512 with 32x128, 16x256, 32x256, 64x128 tiles), A/B twice, then
# each variant's permutation tests.
set -o pipefail
export TMPDIR=/tmp
L=tools/ab_libs
T=r02p
for rep in 1 2; do
timeout -k 10 600 python tools/ab_bench.py $L/lib_base.so $L/lib_f32x128.so $L/lib_f16x256.so $L/lib_f32x256.so $L/lib_f64x128.so --ops c5_T,c5_perm --rounds 5 > gpurun_out/ab_f512_${T}_$rep.log 2>&1 || { echo AB_FAIL; tail -20 gpurun_out/ab_f512_${T}_$rep.log; exit 1; }
grep -v amdgpu.ids gpurun_out/ab_f512_${T}_$rep.log
done
for v in f32x128 f16x256 f32x256 f64x128; do
BOLT_AMD_LIB=$L/lib_$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_fuzz_medium.py "tests/test_gpu_large.py::test_transpose_full_size" -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/f512_tests_${T}_$v.log 2>&1 || { echo TESTS_FAIL $v; tail -30 gpurun_out/f512_tests_${T}_$v.log; exit 1; }
echo $v; tail -1 gpurun_out/f512_tests_${T}_$v.log
done
echo ALL_OK
