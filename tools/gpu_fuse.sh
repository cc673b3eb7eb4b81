set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_large.py -m gpu -q -x -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/fuse_tests.log 2>&1 || { echo TESTS_FAIL; exit 1; }
timeout -k 10 600 python tools/ab_bench.py tools/ab_f0.so tools/ab_f1.so --ops c5_T,c5_perm,c3_T,c2_swap > gpurun_out/ab_fuse.log 2>&1 || { echo AB_FAIL; exit 1; }
echo ALL_OK
