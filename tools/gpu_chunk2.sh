set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_chunk_paths.py tests/test_abi.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/chunk_tests.log 2>&1 || { echo TESTS_FAIL; exit 1; }
BOLT_AMD_RECMAP_PARTS=0 timeout -k 10 300 python tools/chunk_bench.py > gpurun_out/chunk_parts0.log 2>&1 || { echo B0_FAIL; exit 1; }
timeout -k 10 300 python tools/chunk_bench.py > gpurun_out/chunk_parts1.log 2>&1 || { echo B1_FAIL; exit 1; }
BOLT_AMD_RECMAP_PARTS=0 timeout -k 10 300 python tools/chunk_bench.py > gpurun_out/chunk_parts0b.log 2>&1 || { echo B0_FAIL; exit 1; }
timeout -k 10 300 python tools/chunk_bench.py > gpurun_out/chunk_parts1b.log 2>&1 || { echo B1_FAIL; exit 1; }
echo ALL_OK
