# Round re-entry check on a fresh box: full -m gpu suite, smoke, default C2 bench
# (cpu_baseline + PMC traffic), rocprofv3 kernel summary of the same bench.
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_r02a.log 2>&1 || { echo TESTS_FAIL; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r02a.log 2>&1 || { echo SMOKE_FAIL; exit 1; }
timeout -k 10 600 python bench.py > gpurun_out/bench_r02a_c2.json 2> gpurun_out/bench_r02a_c2.err || { echo BENCH_FAIL; exit 1; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r02a_c2 -o run --output-format csv -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-pmc > gpurun_out/prof_r02a_c2.log 2>&1 || { echo PROF_FAIL; exit 1; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r02a_c5 -o run --output-format csv -- python bench.py --config C5 --steps 5 --warmup 2 --no-cpu-baseline --no-pmc > gpurun_out/prof_r02a_c5.log 2>&1 || { echo PROF5_FAIL; exit 1; }
echo ALL_OK
