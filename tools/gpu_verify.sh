# GPU: full -m gpu suite, smoke, C2 bench (+PMC), rocprof of the bench (run under gpurun)
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAIL; exit 1; }
bash tools/gpu_bench_c2.sh
