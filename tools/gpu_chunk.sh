# chunk path verification + A/B of the fused re-chunk (run under gpurun)
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_chunk_paths.py tests/test_gpu_large.py -k "chunk or record or rechunk" -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/chunk_tests.log 2>&1 || { echo TESTS_FAIL; exit 1; }
BOLT_AMD_FUSED_RECHUNK=0 timeout -k 10 300 python tools/chunk_bench.py > gpurun_out/chunk_fused0.log 2>&1 || { echo BENCH0_FAIL; exit 1; }
timeout -k 10 300 python tools/chunk_bench.py > gpurun_out/chunk_fused1.log 2>&1 || { echo BENCH1_FAIL; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_chunk -o run --output-format csv -- python tools/chunk_bench.py > gpurun_out/chunk_prof.log 2>&1 || { echo PROF_FAIL; exit 1; }
echo ALL_OK
