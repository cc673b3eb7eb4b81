set -o pipefail
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAIL; exit 1; }
timeout -k 10 300 python tools/chunk_bench.py > gpurun_out/chunk.log 2>&1 || { echo CHUNK_FAIL; exit 1; }
bash tools/gpu_configs.sh
