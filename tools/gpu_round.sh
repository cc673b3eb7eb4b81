# GPU verification + measurement pass (run from the repo root under gpurun)
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAIL; exit 1; }
if [ -n "$AB_LIBS" ]; then
  timeout -k 10 600 python tools/ab_bench.py $AB_LIBS --ops ${AB_OPS:-c2_swap,c2_mean_rows,c2_std_rows} > gpurun_out/ab.log 2>&1 || { echo AB_FAIL; exit 1; }
fi
timeout -k 10 300 python tools/transfer_bench.py > gpurun_out/transfer.log 2>&1 || { echo TRANSFER_FAIL; exit 1; }
timeout -k 10 300 python tools/chunk_bench.py > gpurun_out/chunk.log 2>&1 || { echo CHUNK_FAIL; exit 1; }
timeout -k 10 300 python tools/index_bench.py > gpurun_out/index.log 2>&1 || { echo INDEX_FAIL; exit 1; }
bash tools/gpu_bench_c2.sh
