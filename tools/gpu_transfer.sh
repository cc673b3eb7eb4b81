set -o pipefail
export TMPDIR=/tmp
for th in 4 8 16; do
  BOLT_AMD_COPY_THREADS=$th timeout -k 10 300 python tools/transfer_bench.py > gpurun_out/transfer_t$th.log 2>&1 || { echo FAIL; exit 1; }
done
BOLT_AMD_COPY_THREADS=8 BOLT_AMD_COPY_CHUNK_MB=16 timeout -k 10 300 python tools/transfer_bench.py > gpurun_out/transfer_t8_c16.log 2>&1 || { echo FAIL; exit 1; }
BOLT_AMD_H2D=direct timeout -k 10 300 python tools/transfer_bench.py > gpurun_out/transfer_direct.log 2>&1 || { echo FAIL; exit 1; }
echo ALL_OK
