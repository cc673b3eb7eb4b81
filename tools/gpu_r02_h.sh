# Round 2: f64 square tiles for C5 .T (512-B source segments) and the
# values_to_keys part budget, A/B in one process; the square-tile build's
# correctness on the permutation / large tests.
set -o pipefail
export TMPDIR=/tmp
L=tools/ab_libs
timeout -k 10 600 python tools/ab_bench.py $L/lib_base.so $L/lib_t8sq.so --ops c5_T,c5_perm,c5_T,c5_pack,c5_v2k,c5_v2k_pb16k,c5_v2k_pb24k --rounds 7 > gpurun_out/ab_t8_r02h.log 2>&1 || { echo AB_FAIL; tail -20 gpurun_out/ab_t8_r02h.log; exit 1; }
grep -v amdgpu.ids gpurun_out/ab_t8_r02h.log
BOLT_AMD_LIB=$L/lib_t8sq.so timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_fuzz_medium.py "tests/test_gpu_large.py::test_transpose_full_size" -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/t8_tests_r02h.log 2>&1 || { echo TESTS_FAIL; tail -30 gpurun_out/t8_tests_r02h.log; exit 1; }
tail -2 gpurun_out/t8_tests_r02h.log
echo ALL_OK
