# Round 2: software-pipelined packed (1-/2-byte) transposes (BM_PK_PIPE: next
# tile's loads in flight during the current tile's stores; 1, 2, 4 blocks per
# CU of grid), A/B twice, then each variant's permutation tests.
set -o pipefail
export TMPDIR=/tmp
L=tools/ab_libs
T=r02u
for rep in 1 2; do
timeout -k 10 600 python tools/ab_bench.py $L/lib_base.so $L/lib_p1.so $L/lib_p2.so $L/lib_p4.so --ops u16_T,u8_T,u16_2d,c2_swap --rounds 5 > gpurun_out/ab_${T}_$rep.log 2>&1 || { echo AB_FAIL; tail -20 gpurun_out/ab_${T}_$rep.log; exit 1; }
grep -v amdgpu.ids gpurun_out/ab_${T}_$rep.log
done
for v in p1 p2 p4; do
BOLT_AMD_LIB=$L/lib_$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_fuzz_medium.py "tests/test_gpu_large.py::test_transpose_full_size" -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/tests_${T}_$v.log 2>&1 || { echo TESTS_FAIL $v; tail -30 gpurun_out/tests_${T}_$v.log; exit 1; }
echo $v; tail -1 gpurun_out/tests_${T}_$v.log
done
echo ALL_OK
