set -o pipefail
export TMPDIR=/tmp
for i in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-pmc > gpurun_out/r9_c2_$i.json 2> gpurun_out/r9_c2.err || { echo BENCH_FAIL; exit 1; }
done
bash tools/gpu_configs_prof.sh r9 C3 C4
