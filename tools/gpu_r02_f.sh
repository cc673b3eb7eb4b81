# Round 2: L2-conflict experiments.  (1) diagonal-walk A/B of the product
# kernels (lib_base vs tile/row skew builds, one process, interleaved);
# (2) the diagonal rowcopy microbench at full C3 size; (3) the skew builds'
# correctness (every 4-d permutation kernel test + full-size C3/C5 parity);
# (4) egress variants for toarray; (5) XCD-contiguous rows for k_red_rows
# (time A/B + FETCH_SIZE on 8000-B rows).
set -o pipefail
export TMPDIR=/tmp
L=tools/ab_libs
timeout -k 10 600 python tools/ab_bench.py $L/lib_base.so $L/lib_trskew.so $L/lib_rcskew.so $L/lib_both.so --ops c5_T,c5_perm,c2_swap,c3_full,c3_T,c4_full,u16_T,t64_swap --rounds 5 > gpurun_out/ab_skew_r02f.log 2>&1 || { echo AB_FAIL; tail -20 gpurun_out/ab_skew_r02f.log; exit 1; }
cat gpurun_out/ab_skew_r02f.log
timeout -k 10 120 /opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -o /tmp/rcs.bin tools/skew/rowcopy_skew.hip > /dev/null 2>&1 || { echo BUILD_FAIL; exit 1; }
timeout -k 10 300 /tmp/rcs.bin > gpurun_out/rcs_r02f.log 2>&1 || { echo RCS_FAIL; tail gpurun_out/rcs_r02f.log; exit 1; }
cat gpurun_out/rcs_r02f.log
BOLT_AMD_LIB=$L/lib_both.so timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_fuzz_medium.py "tests/test_gpu_large.py::test_swap_full_size" "tests/test_gpu_large.py::test_transpose_full_size" -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/skew_tests_r02f.log 2>&1 || { echo SKEW_TESTS_FAIL; tail -30 gpurun_out/skew_tests_r02f.log; exit 1; }
tail -2 gpurun_out/skew_tests_r02f.log
timeout -k 10 300 python tools/egress_probe.py > gpurun_out/egress_r02f.log 2>&1 || { echo EGRESS_FAIL; tail gpurun_out/egress_r02f.log; exit 1; }
cat gpurun_out/egress_r02f.log
timeout -k 10 300 python tools/ab_bench.py $L/lib_base.so $L/lib_redxcd.so --ops c2_mean_rows,c2_std_rows --rounds 7 > gpurun_out/ab_redxcd_r02f.log 2>&1 || { echo AB2_FAIL; exit 1; }
cat gpurun_out/ab_redxcd_r02f.log
BOLT_AMD_LIB=$L/lib_redxcd.so timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_redxcd -o pmc --output-format csv -- python tools/reduce_align.py > gpurun_out/pmc_redxcd.log 2>&1 || { echo PMC_FAIL; exit 1; }
echo ALL_OK
