set -o pipefail
for i in 1 2 3 4; do
  timeout -k 10 120 python tools/host_ab.py .ab_old || exit 1
  timeout -k 10 120 python tools/host_ab.py . || exit 1
done
