# bm_stream_wait A/B: sync probe, GPU test suite, C2 bench
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python tools/sync_probe.py > gpurun_out/sync_probe.log 2>&1 || { echo PROBE_FAIL; exit 1; }
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/gpu_tests8.log 2>&1 || { echo TESTS_FAIL; exit 1; }
timeout -k 10 300 python bench.py --no-cpu-baseline --no-pmc > gpurun_out/bench8_c2.json 2> gpurun_out/bench8_c2.err || { echo BENCH_FAIL; exit 1; }
BOLT_AMD_SPIN_US=0 timeout -k 10 300 python bench.py --no-cpu-baseline --no-pmc > gpurun_out/bench8_c2_nospin.json 2>> gpurun_out/bench8_c2.err || { echo BENCH_FAIL; exit 1; }
timeout -k 10 300 python bench.py --no-cpu-baseline --no-pmc > gpurun_out/bench8_c2_b.json 2>> gpurun_out/bench8_c2.err || { echo BENCH_FAIL; exit 1; }
echo ALL_OK
