set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/all_axes_padded_probe.py > gpurun_out/r06za_all_axes.log 2>&1 || { echo FAIL; tail -20 gpurun_out/r06za_all_axes.log; exit 1; }
cat gpurun_out/r06za_all_axes.log
echo ALL_OK
