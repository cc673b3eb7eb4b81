# Every BASELINE config on one GPU: full bench line (PMC traffic + CPU baseline)
# and a rocprofv3 --kernel-trace --stats summary of the same step.
# usage: bash tools/gpu_configs_prof.sh TAG CONFIG...
set -o pipefail
export TMPDIR=/tmp
tag=$1; shift
for c in "$@"; do
  echo "bench $c"
  timeout -k 10 400 python bench.py --config $c --steps 5 --warmup 1 > gpurun_out/${tag}_$c.json 2> gpurun_out/${tag}_$c.err || { echo "BENCH_FAIL $c"; exit 1; }
  echo "rocprof $c"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_prof_$c -o run --output-format csv -- python bench.py --config $c --steps 5 --warmup 1 --no-cpu-baseline --no-pmc > gpurun_out/${tag}_prof_$c.log 2>&1 || { echo "PROF_FAIL $c"; exit 1; }
done
echo ALL_OK
