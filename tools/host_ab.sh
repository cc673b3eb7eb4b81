# Host-path A/B of the C2 step, old tree vs this one, in alternating fresh
# processes on one GPU (tools/host_ab.py).  Before the gpurun call, put the
# old package next to this tree:
#   mkdir -p .ab_old && git archive <ref> bolt_amd | tar -x -C .ab_old
# (.ab_old is git-ignored; it uses this tree's libbolt_mi355x.so).
set -o pipefail
for i in 1 2 3 4; do
  timeout -k 10 120 python tools/host_ab.py .ab_old || exit 1
  timeout -k 10 120 python tools/host_ab.py . || exit 1
done
