set -o pipefail
export TMPDIR=/tmp
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-pmc > gpurun_out/r10_c2_$i.json 2> gpurun_out/r10_c2.err || { echo BENCH_FAIL; exit 1; }
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r10_prof_c2 -o run --output-format csv -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-pmc > gpurun_out/r10_prof_c2.log 2>&1 || { echo PROF_FAIL; exit 1; }
echo ALL_OK
