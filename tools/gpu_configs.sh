set -o pipefail
export TMPDIR=/tmp
for c in C3 C4 C5 target64; do
  timeout -k 10 600 python bench.py --config $c --steps 5 --warmup 1 --no-cpu-baseline --no-pmc > gpurun_out/bench_$c.json 2> gpurun_out/bench_$c.err || { echo "BENCH_FAIL $c"; exit 1; }
done
# (rocprof of C3: tools/gpu_round*.sh)
echo ALL_OK
