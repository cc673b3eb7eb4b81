# C5 bench (the chunk pack runs bm_record_gather) + the chunk parity tests.
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_chunk_paths.py tests/test_fuzz_oracle.py -m gpu -q -x \
  -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/c5_tests.log 2>&1 || { echo TEST_FAIL; exit 1; }
timeout -k 10 600 python bench.py --config C5 --steps 5 --warmup 1 --no-cpu-baseline --no-pmc > gpurun_out/bench_C5.json 2> gpurun_out/bench_C5.err || { echo BENCH_FAIL; exit 1; }
timeout -k 10 600 python tools/chunk_bench.py > gpurun_out/chunk.log 2>&1 || { echo CHUNK_FAIL; exit 1; }
echo ALL_OK
