# Fuzz soak on one GPU: the seeded oracle and medium-size fuzz cases over
# seed ranges beyond the suite's (BOLT_AMD_FUZZ_SEEDS), stopping at the first
# failure.  ORACLE=start:stop MEDIUM=start:stop TAG=r05j bash tools/gpu_fuzz_soak.sh
set -o pipefail
T=${TAG:-soak}
mkdir -p gpurun_out
echo "[$(date +%T)] oracle fuzz ${ORACLE:-200:1200}"
BOLT_AMD_FUZZ_SEEDS=${ORACLE:-200:1200} timeout -k 10 900 python -u -m pytest tests/test_fuzz_oracle.py -m gpu -x -q \
  --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_fuzz_oracle.log 2>&1 \
  || { echo ORACLE_FUZZ_FAIL; tail -40 gpurun_out/${T}_fuzz_oracle.log; exit 1; }
tail -1 gpurun_out/${T}_fuzz_oracle.log
echo "[$(date +%T)] medium fuzz ${MEDIUM:-240:1240}"
BOLT_AMD_FUZZ_SEEDS=${MEDIUM:-240:1240} timeout -k 10 900 python -u -m pytest tests/test_gpu_fuzz_medium.py -m gpu -x -q \
  --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_fuzz_medium.log 2>&1 \
  || { echo MEDIUM_FUZZ_FAIL; tail -40 gpurun_out/${T}_fuzz_medium.log; exit 1; }
tail -1 gpurun_out/${T}_fuzz_medium.log
echo ALL_OK
