# Fuzz soak on one GPU: the seeded fuzz suites over seed ranges beyond the
# suite's (BOLT_AMD_FUZZ_SEEDS; the padded-row variants of tests/test_row_pitch.py:
# BOLT_AMD_PITCH_SEEDS), each stopping at its first failure.  ONLY="padded api"
# runs a subset.
#   TAG=r05j ORACLE=200:2200 MEDIUM=240:1240 GETITEM=300:3300 API=200:1200 CHUNK=200:1200 PADDED=60:1060 bash tools/gpu_fuzz_soak.sh
set -o pipefail
T=${TAG:-soak}
mkdir -p gpurun_out
want() { [ -z "$ONLY" ] && return 0; case " $ONLY " in *" $1 "*) return 0;; esac; return 1; }
run() {  # name test-file seeds [seed variable]
  want $1 || return 0
  echo "[$(date +%T)] $1 fuzz $3"
  env ${4:-BOLT_AMD_FUZZ_SEEDS}=$3 timeout -k 10 900 python -u -m pytest $2 -m gpu -x -q \
    --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_fuzz_$1.log 2>&1 \
    || { echo "$1 FUZZ_FAIL"; tail -40 gpurun_out/${T}_fuzz_$1.log; return 1; }
  tail -1 gpurun_out/${T}_fuzz_$1.log
}
run oracle tests/test_fuzz_oracle.py ${ORACLE:-200:1200} &&
run medium tests/test_gpu_fuzz_medium.py ${MEDIUM:-240:1240} &&
run getitem tests/test_getitem_fuzz.py ${GETITEM:-300:3300} &&
run api tests/test_api_fuzz.py ${API:-200:1200} &&
run chunk tests/test_chunk_fuzz.py ${CHUNK:-200:1200} &&
run padded tests/test_row_pitch.py ${PADDED:-60:1060} BOLT_AMD_PITCH_SEEDS &&
echo ALL_OK
