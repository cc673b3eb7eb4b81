# A/B of the C2 step (swap + mean + std, tools/host_ab.py) with the swap's
# result stored at a padded row pitch (BOLT_AMD_ROW_PITCH=1, the default)
# against dense rows (=0), in alternating fresh processes on one GPU.
set -o pipefail
for i in 1 2 3 4; do
  BOLT_AMD_ROW_PITCH=0 timeout -k 10 120 python tools/host_ab.py . || exit 1
  BOLT_AMD_ROW_PITCH=1 timeout -k 10 120 python tools/host_ab.py . || exit 1
done
