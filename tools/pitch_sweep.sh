# Row-pitch sweep of the C2 step (tools/host_ab.py) under rocprofv3
# --kernel-trace --stats: the swap's transpose and the two row statistics at
# each destination pitch (bytes = align-up + skew; 8000 = dense).  Read the
# per-kernel times with tools/rocpd_stats.py gpurun_out/${T}_*/run_results.db.
set -o pipefail
T=${T:-r05t}
export TMPDIR=/tmp
run() {  # tag, then env assignments
  tag=$1; shift
  env "$@" timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_$tag -o run -- \
      python tools/host_ab.py . 3 20 > gpurun_out/${T}_$tag.log 2>&1 || exit 1
}
run dense BOLT_AMD_ROW_PITCH=0
run p8064 BOLT_AMD_PITCH_ALIGN=128 BOLT_AMD_PITCH_PAD_DIV=4
run p8192 BOLT_AMD_PITCH_ALIGN=1024 BOLT_AMD_PITCH_PAD_DIV=4
run p8320 BOLT_AMD_PITCH_ALIGN=1024 BOLT_AMD_PITCH_SKEW=128 BOLT_AMD_PITCH_PAD_DIV=4
run p8448 BOLT_AMD_PITCH_ALIGN=1024 BOLT_AMD_PITCH_SKEW=256 BOLT_AMD_PITCH_PAD_DIV=4
run p8704 BOLT_AMD_PITCH_ALIGN=1024 BOLT_AMD_PITCH_SKEW=512 BOLT_AMD_PITCH_PAD_DIV=4
run p9216 BOLT_AMD_PITCH_ALIGN=1024 BOLT_AMD_PITCH_SKEW=1024 BOLT_AMD_PITCH_PAD_DIV=4
run p8192b BOLT_AMD_PITCH_ALIGN=1024 BOLT_AMD_PITCH_PAD_DIV=4
