# Round 6 checkpoint on the final kernels (rows reduction with whole
# wave-wide steps): GPU suite, smoke, the default bench, the same bench under
# rocprofv3 --kernel-trace --stats (summary + per-kernel table), and the
# N-rank rehearsal at 2 and 4 ranks on one GPU.
set -o pipefail
export TMPDIR=/tmp
T=${TAG:-r06m}
TAG=$T NS="2 4" bash tools/gpu_r05_checkpoint.sh || exit 1
python tools/trace_stats.py gpurun_out/${T}_prof/run_kernel_trace.csv --match k_ > gpurun_out/${T}_trace_stats.txt 2>&1 || true
ls gpurun_out/${T}_prof/
head -40 gpurun_out/${T}_trace_stats.txt
echo ALL_OK
