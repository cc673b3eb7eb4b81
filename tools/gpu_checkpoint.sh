# Checkpoint on one MI355X: the whole -m gpu suite, smoke, the default bench
# (C2 + 64 GiB target sub-record, PMC traffic, CPU baselines), the C1 line,
# and C3 / C4 / C5 bench lines with their rocprofv3 kernel summaries.
#   TAG=r03x bash tools/gpu_checkpoint.sh            (outputs gpurun_out/*_$TAG*)
#   SKIP_TESTS=1 ... to skip the test suite; CONFIGS="C3 C5" to choose configs
set -o pipefail
export TMPDIR=/tmp
T=${TAG:-r03}
CONFIGS=${CONFIGS:-"C3 C4 C5"}
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q --maxfail=30 -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_$T.log 2>&1 || { echo TESTS_FAIL; tail -40 gpurun_out/gpu_tests_$T.log; exit 1; }
  tail -2 gpurun_out/gpu_tests_$T.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$T.log 2>&1 || { echo SMOKE_FAIL; tail gpurun_out/smoke_$T.log; exit 1; }
  cat gpurun_out/smoke_$T.log
fi
timeout -k 10 900 python bench.py > gpurun_out/bench_${T}_C2.json 2> gpurun_out/bench_${T}_C2.err || { echo BENCH_FAIL; tail gpurun_out/bench_${T}_C2.err; exit 1; }
cat gpurun_out/bench_${T}_C2.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${T}_C2 -o run --output-format csv -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-pmc --no-target64 > gpurun_out/prof_${T}_C2.log 2>&1 || { echo PROF_FAIL; exit 1; }
timeout -k 10 600 python bench.py --config C1 > gpurun_out/bench_${T}_C1.json 2> gpurun_out/bench_${T}_C1.err || { echo BENCH_C1_FAIL; tail gpurun_out/bench_${T}_C1.err; exit 1; }
cat gpurun_out/bench_${T}_C1.json
for c in $CONFIGS; do
  timeout -k 10 900 python bench.py --config $c --steps 5 --warmup 1 > gpurun_out/bench_${T}_$c.json 2> gpurun_out/bench_${T}_$c.err || { echo BENCH_${c}_FAIL; tail gpurun_out/bench_${T}_$c.err; exit 1; }
  cat gpurun_out/bench_${T}_$c.json
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${T}_$c -o run --output-format csv -- python bench.py --config $c --steps 5 --warmup 1 --no-cpu-baseline --no-pmc > gpurun_out/prof_${T}_$c.log 2>&1 || { echo PROF_${c}_FAIL; exit 1; }
done
echo ALL_OK
