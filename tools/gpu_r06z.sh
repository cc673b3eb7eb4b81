# Round 6, call z: mean / var / std over every axis of a row-padded float
# array read in place (array.py _padded_all_moments): the row-pitch and
# full-size GPU tests, then the whole GPU suite and smoke.
set -o pipefail
export TMPDIR=/tmp
T=${TAG:-r06z}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_row_pitch.py tests/test_gpu_large.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_focus.log 2>&1 || { echo FOCUS_FAIL; tail -30 gpurun_out/${T}_focus.log; exit 1; }
tail -1 gpurun_out/${T}_focus.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_gpu_tests.log 2>&1 || { echo TESTS_FAIL; tail -30 gpurun_out/${T}_gpu_tests.log; exit 1; }
tail -1 gpurun_out/${T}_gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 gpurun_out/${T}_smoke.log; exit 1; }
tail -1 gpurun_out/${T}_smoke.log
echo ALL_OK
