# Same-box comparison: the product's C5 .T (ab_bench, hipEvents) beside the
# standalone tile kernels of tools/microbench/transpose_c5t.hip
set -o pipefail
export TMPDIR=/tmp
hipcc -O3 -std=c++17 --offload-arch=gfx950 -o tools/microbench/tc5t.bin tools/microbench/transpose_c5t.hip -ldl || exit 1
timeout -k 10 300 ./tools/microbench/tc5t.bin bolt_amd/libbolt_mi355x.so > gpurun_out/r02_ab_c5t_b.log 2>&1 || { echo C5T_FAIL; tail gpurun_out/r02_ab_c5t_b.log; exit 1; }
cat gpurun_out/r02_ab_c5t_b.log
