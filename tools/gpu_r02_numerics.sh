# Round 2: batched-Welford var/std + ufunc reduce modes on the GPU: full -m gpu
# suite (new numerics / reduce / reshape fixtures), smoke, C2 bench and its
# rocprofv3 kernel summary (reduction kernel time after the numerics change).
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --maxfail=30 -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_r02b.log 2>&1 || { echo TESTS_FAIL; tail -30 gpurun_out/gpu_tests_r02b.log; exit 1; }
tail -3 gpurun_out/gpu_tests_r02b.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r02b.log 2>&1 || { echo SMOKE_FAIL; exit 1; }
timeout -k 10 600 python bench.py --no-pmc > gpurun_out/bench_r02b_c2.json 2> gpurun_out/bench_r02b_c2.err || { echo BENCH_FAIL; exit 1; }
cat gpurun_out/bench_r02b_c2.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r02b_c2 -o run --output-format csv -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-pmc > gpurun_out/prof_r02b_c2.log 2>&1 || { echo PROF_FAIL; exit 1; }
echo ALL_OK
