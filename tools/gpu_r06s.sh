# Round 6, call s: k_recmap_reg (map entries in registers, one record per
# tile) against the shipped k_recmap_lds: the chunk GPU tests, byte identity
# over three placements, then interleaved timing beside each placement's copy.
set -o pipefail
export TMPDIR=/tmp
T=${TAG:-r06s}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_chunk_paths.py tests/test_chunk_fuzz.py tests/test_golden_api.py > gpurun_out/${T}_tests.log 2>&1 || { echo TESTS_FAIL; tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -2 gpurun_out/${T}_tests.log
timeout -k 10 500 python -u tools/dst_placement_ab.py tools/ab_libs/pack_base.so tools/ab_libs/pack_reg.so --ops c5_pack,c5_pack_copy --k 3 --rounds 3 --reps 3 --check > gpurun_out/${T}_ab.log 2>&1 || { echo AB_FAIL; tail -20 gpurun_out/${T}_ab.log; exit 1; }
cat gpurun_out/${T}_ab.log
timeout -k 10 200 python -u tools/ab_bench.py tools/ab_libs/pack_base.so tools/ab_libs/pack_reg.so --ops c5_pack --rounds 7 --reps 5 > gpurun_out/${T}_ab2.log 2>&1 || { echo AB2_FAIL; tail -20 gpurun_out/${T}_ab2.log; exit 1; }
cat gpurun_out/${T}_ab2.log
echo ALL_OK
