# Round 6, call w: egress rates on the final tree -- the dense staged path
# (tools/egress_probe.py) and toarray() of C2's row-padded swap result
# against a dense array of the same bytes (tools/egress_padded_probe.py).
set -o pipefail
export TMPDIR=/tmp
T=${TAG:-r06w}
mkdir -p gpurun_out
(cat /sys/kernel/mm/transparent_hugepage/enabled 2>&1 || true) > gpurun_out/${T}_thp.txt
timeout -k 10 300 python -u tools/egress_padded_probe.py > gpurun_out/${T}_egress_padded.log 2>&1 || { echo PAD_FAIL; tail -20 gpurun_out/${T}_egress_padded.log; exit 1; }
cat gpurun_out/${T}_egress_padded.log
timeout -k 10 300 python -u tools/egress_probe.py > gpurun_out/${T}_egress.log 2>&1 || { echo EG_FAIL; tail -20 gpurun_out/${T}_egress.log; exit 1; }
cat gpurun_out/${T}_egress.log gpurun_out/${T}_thp.txt
echo ALL_OK
