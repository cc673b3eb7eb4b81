set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAIL; exit 1; }
timeout -k 10 600 python bench.py --steps 20 --warmup 3 > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err || { echo BENCH_FAIL; exit 1; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c2 -o run --output-format csv -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-pmc > gpurun_out/prof_c2.log 2>&1 || { echo PROF_FAIL; exit 1; }
echo ALL_OK
