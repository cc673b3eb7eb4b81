# Host wait policy on the C2 step: runtime synchronize vs hipStreamQuery spin (C / torch), one process
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python tools/sync_spin_probe.py > gpurun_out/r02_sync_spin.log 2>&1 || { echo PROBE_FAIL; tail -20 gpurun_out/r02_sync_spin.log; exit 1; }
cat gpurun_out/r02_sync_spin.log
