# A/B of the record-map gather's staging / gather batching (tools/ab_*.so built
# with -DBM_STAGE_U / -DBM_GATHER_U), then the record-map parity tests on the
# in-tree build.
set -o pipefail
export TMPDIR=/tmp
#timeout -k 10 300 python -u -m pytest tests/test_chunk_paths.py tests/test_gpu_kernels.py -m gpu -q -x \
#  -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/recmap_tests.log 2>&1 || { echo TEST_FAIL; exit 1; }
timeout -k 10 600 python tools/ab_bench.py tools/ab_old.so tools/ab_new.so tools/ab_s4.so \
  --ops c5_pack_whole,c5_pack,c5_v2k_whole,c5_v2k > gpurun_out/ab_recmap.log 2>&1 || { echo AB_FAIL; exit 1; }
echo ALL_OK
