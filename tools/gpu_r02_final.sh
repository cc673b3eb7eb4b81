# Round 2 final tree: whole -m gpu suite, smoke, default bench (C2 + 64 GiB target, PMC, CPU baseline)
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --maxfail=30 -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_r02f.log 2>&1 || { echo TESTS_FAIL; tail -40 gpurun_out/gpu_tests_r02f.log; exit 1; }
tail -2 gpurun_out/gpu_tests_r02f.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r02f.log 2>&1 || { echo SMOKE_FAIL; tail gpurun_out/smoke_r02f.log; exit 1; }
cat gpurun_out/smoke_r02f.log
timeout -k 10 900 python bench.py > gpurun_out/bench_r02f_c2.json 2> gpurun_out/bench_r02f_c2.err || { echo BENCH_FAIL; tail gpurun_out/bench_r02f_c2.err; exit 1; }
cat gpurun_out/bench_r02f_c2.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r02f_c2 -o run --output-format csv -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-pmc --no-target64 > gpurun_out/prof_r02f_c2.log 2>&1 || { echo PROF_FAIL; exit 1; }
echo ALL_OK
