set -o pipefail
export TMPDIR=/tmp
for c in C3 C4 C5 target64; do
  timeout -k 10 600 python bench.py --config $c --steps 5 --warmup 1 --no-cpu-baseline --no-pmc > gpurun_out/bench_$c.json 2> gpurun_out/bench_$c.err || { echo "BENCH_FAIL $c"; exit 1; }
done
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_cfg -o run --output-format csv -- python bench.py --config C3 --steps 3 --warmup 1 --no-cpu-baseline --no-pmc > gpurun_out/prof_cfg.log 2>&1 || { echo PROF_FAIL; exit 1; }
echo ALL_OK
