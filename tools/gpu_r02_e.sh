# Round 2: limiter counters of the sub-0.72 kernels + reduction over-fetch attribution.
set -o pipefail
export TMPDIR=/tmp
bash tools/gpu_kernel_counters.sh || exit 1
bash tools/gpu_pmc_reduce_align.sh || exit 1
echo ALL_OK
