# Direct-to-LDS staging A/B of the f32 tile transpose:
# register staging (the product's structure) vs global_load_lds variants.
set -o pipefail
export TMPDIR=/tmp
cd tools/microbench
hipcc -O3 -std=c++17 --offload-arch=gfx950 -o tglds.bin transpose_glds.hip || exit 1
cd ../..
timeout -k 10 300 ./tools/microbench/tglds.bin > gpurun_out/r02_ab_glds.log 2>&1 || { echo GLDS_FAIL; tail gpurun_out/r02_ab_glds.log; exit 1; }
cat gpurun_out/r02_ab_glds.log
