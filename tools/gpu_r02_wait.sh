# A/B of the host's wait policy on the C2 step: the HIP runtime's default
# (active wait ROC_ACTIVE_WAIT_TIMEOUT, then an interrupt) vs a longer active
# wait, alternated in fresh processes.
set -o pipefail
export TMPDIR=/tmp
for i in 1 2 3; do
  for w in default 2000 100000; do
    if [ $w = default ]; then
      timeout -k 10 300 python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-pmc --no-target64 > gpurun_out/wait_${w}_$i.json 2>/dev/null || { echo FAIL; exit 1; }
    else
      ROC_ACTIVE_WAIT_TIMEOUT=$w timeout -k 10 300 python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-pmc --no-target64 > gpurun_out/wait_${w}_$i.json 2>/dev/null || { echo FAIL; exit 1; }
    fi
    python -c "import json; d=json.load(open('gpurun_out/wait_${w}_$i.json')); print('$w', '$i', d['value'], d['ms_per_step'], d['roofline']['avg_ms'])"
  done
done
