# Round 2: per-block page-local batch walk for transposes (BM_TR_LOOP) A/B,
# its correctness on the permutation tests, then the default bench and the
# C3 line with the 16x16 diagonal rowcopy now on by default.
set -o pipefail
export TMPDIR=/tmp
L=tools/ab_libs
T=r02n
for rep in 1 2; do
timeout -k 10 600 python tools/ab_bench.py $L/lib_base.so $L/lib_loop.so --ops c5_T,c5_perm,c3_T,u16_T,u8_T,c2_swap --rounds 5 > gpurun_out/ab_loop_${T}_$rep.log 2>&1 || { echo AB_FAIL; tail -20 gpurun_out/ab_loop_${T}_$rep.log; exit 1; }
grep -v amdgpu.ids gpurun_out/ab_loop_${T}_$rep.log
done
BOLT_AMD_LIB=$L/lib_loop.so timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_fuzz_medium.py "tests/test_gpu_large.py::test_transpose_full_size" -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/loop_tests_$T.log 2>&1 || { echo TESTS_FAIL; tail -30 gpurun_out/loop_tests_$T.log; exit 1; }
tail -2 gpurun_out/loop_tests_$T.log
timeout -k 10 900 python bench.py > gpurun_out/bench_${T}_c2.json 2> gpurun_out/bench_${T}_c2.err || { echo BENCH_FAIL; tail gpurun_out/bench_${T}_c2.err; exit 1; }
cat gpurun_out/bench_${T}_c2.json
timeout -k 10 900 python bench.py --config C3 --steps 5 --warmup 1 > gpurun_out/bench_${T}_C3.json 2> gpurun_out/bench_${T}_C3.err || { echo BENCH_C3_FAIL; tail gpurun_out/bench_${T}_C3.err; exit 1; }
cat gpurun_out/bench_${T}_C3.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${T}_C3 -o run --output-format csv -- python bench.py --config C3 --steps 5 --warmup 1 --no-cpu-baseline --no-pmc > gpurun_out/prof_${T}_C3.log 2>&1 || { echo PROF_C3_FAIL; exit 1; }
echo ALL_OK
