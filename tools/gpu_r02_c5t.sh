# C5 .T tile-order / pipelined-block A/B (tools/microbench/transpose_c5t.hip)
set -o pipefail
export TMPDIR=/tmp
hipcc -O3 -std=c++17 --offload-arch=gfx950 -o tools/microbench/tc5t.bin tools/microbench/transpose_c5t.hip || exit 1
timeout -k 10 300 ./tools/microbench/tc5t.bin > gpurun_out/r02_ab_c5t.log 2>&1 || { echo C5T_FAIL; tail gpurun_out/r02_ab_c5t.log; exit 1; }
cat gpurun_out/r02_ab_c5t.log
