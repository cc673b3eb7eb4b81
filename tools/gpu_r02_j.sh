# Round 2: dynamic-LDS column reductions (occupancy of the one-phase case)
# A/B against the static-LDS build; reduction correctness; the LDS record-tile
# transpose microbench for the C3 swap.
set -o pipefail
export TMPDIR=/tmp
L=tools/ab_libs
timeout -k 10 600 python tools/ab_bench.py $L/lib_base.so $L/lib_dyn.so --ops c4_var_cols,t64_std_cols,t64_mean_cols,c2_std_cols,c2_mean_cols,c2_std_rows --rounds 7 > gpurun_out/ab_dyn_r02j.log 2>&1 || { echo AB_FAIL; tail -20 gpurun_out/ab_dyn_r02j.log; exit 1; }
grep -v amdgpu.ids gpurun_out/ab_dyn_r02j.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_numerics.py tests/test_golden_api.py tests/test_gpu_kernels.py "tests/test_gpu_large.py::test_stats_full_size_c4_var" "tests/test_gpu_large.py::test_stats_full_size_c2" -m gpu -q -k "stat or reduce or numerics or full_size" -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/dyn_tests_r02j.log 2>&1 || { echo TESTS_FAIL; tail -30 gpurun_out/dyn_tests_r02j.log; exit 1; }
tail -2 gpurun_out/dyn_tests_r02j.log
timeout -k 10 120 /opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -o /tmp/rcs.bin tools/skew/rowcopy_skew.hip > /dev/null 2>&1 || { echo BUILD_FAIL; exit 1; }
timeout -k 10 300 /tmp/rcs.bin > gpurun_out/rcs_r02j.log 2>&1 || { echo RCS_FAIL; tail gpurun_out/rcs_r02j.log; exit 1; }
cat gpurun_out/rcs_r02j.log
echo ALL_OK
