# C2 default-step repeatability on one box: three bench runs in fresh processes (no PMC / CPU baseline / target64)
set -o pipefail
export TMPDIR=/tmp
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --no-pmc --no-cpu-baseline --no-target64 > gpurun_out/r02_c2rep_$i.json 2> gpurun_out/r02_c2rep_$i.err || { echo BENCH_FAIL; tail gpurun_out/r02_c2rep_$i.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r02_c2rep_$i.json'));print('run $i', d['value'], d['ms_per_step'], d['roofline']['avg_ms'])"
done
