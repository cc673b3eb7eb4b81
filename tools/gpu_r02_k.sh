# Round 2: exact integer var / std for 1-2 byte inputs (C4) -- A/B against
# the float64 Welford path, correctness (numerics incl. exact-rational check,
# stat goldens, full-size C4 var).
set -o pipefail
export TMPDIR=/tmp
L=tools/ab_libs
timeout -k 10 600 python tools/ab_bench.py $L/lib_dyn.so $L/lib_int.so $L/lib_int8.so $L/lib_intblk.so --ops c4_var_full,c4_var_cols,u16_var_rows,t64_std_cols --rounds 7 > gpurun_out/ab_int_r02k.log 2>&1 || { echo AB_FAIL; tail -20 gpurun_out/ab_int_r02k.log; exit 1; }
grep -v amdgpu.ids gpurun_out/ab_int_r02k.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_numerics.py tests/test_golden_api.py tests/test_gpu_kernels.py tests/test_api.py "tests/test_gpu_large.py::test_stats_full_size_c4_var" -m gpu -q -k "stat or reduce or numerics or full_size or int or var" -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/int_tests_r02k.log 2>&1 || { echo TESTS_FAIL; tail -30 gpurun_out/int_tests_r02k.log; exit 1; }
tail -2 gpurun_out/int_tests_r02k.log
echo ALL_OK
