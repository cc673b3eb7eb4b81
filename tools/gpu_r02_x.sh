# Round 2: block-per-output combine for few-output reductions (k_red_combine_blk):
# the reduction tests, the golden statistics / reduce fixtures, the numerics
# tests, then the C1 host-path probe and the C1 bench line.
set -o pipefail
export TMPDIR=/tmp
T=r02x
timeout -k 10 900 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_numerics.py tests/test_golden_api.py -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/tests_$T.log 2>&1 || { echo TESTS_FAIL; tail -40 gpurun_out/tests_$T.log; exit 1; }
tail -1 gpurun_out/tests_$T.log
timeout -k 10 300 python tools/c1_probe.py > gpurun_out/c1_probe_$T.log 2>&1 || { echo PROBE_FAIL; tail gpurun_out/c1_probe_$T.log; exit 1; }
head -12 gpurun_out/c1_probe_$T.log
timeout -k 10 600 python bench.py --config C1 > gpurun_out/bench_${T}_c1.json 2> gpurun_out/bench_${T}_c1.err || { echo BENCH_C1_FAIL; tail gpurun_out/bench_${T}_c1.err; exit 1; }
cat gpurun_out/bench_${T}_c1.json
echo ALL_OK
