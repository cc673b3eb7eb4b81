# index bench + C2 bench/profile (run from the repo root under gpurun)
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python tools/index_bench.py > gpurun_out/index.log 2>&1 || { echo INDEX_FAIL; exit 1; }
bash tools/gpu_bench_c2.sh
