set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 ./tools/microbench/rt.bin > gpurun_out/rt1.log 2>&1 || { echo RT_FAIL; exit 1; }
timeout -k 10 300 python tools/host_overhead.py > gpurun_out/host_ovh.log 2>&1 || { echo HOST_FAIL; exit 1; }
timeout -k 10 600 python bench.py --steps 20 --warmup 3 --no-pmc --no-cpu-baseline > gpurun_out/bench_c2_quick.json 2> gpurun_out/bench_c2_quick.err || { echo BENCH_FAIL; exit 1; }
bash tools/gpu_configs.sh
