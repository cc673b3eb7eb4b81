# Round-5 first check of the reworked bench on one GPU: the default run (C2 +
# stats + target64 + strong C1/C3/C4/C5 sub-records, every op checked, PMC,
# CPU baseline on the whole C2), then the N-rank path rehearsed on one GPU
# with rank 0 under rocprofv3 (gloo host-staged exchanges).
#   TAG=r05a bash tools/gpu_r05_bench_check.sh
set -o pipefail
export TMPDIR=/tmp
T=${TAG:-r05a}
mkdir -p gpurun_out
echo "[$(date +%T)] bench (default run)"
timeout -k 10 900 python bench.py --detail gpurun_out/${T}_bench_detail.json > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { echo BENCH_FAIL; tail -30 gpurun_out/${T}_bench.err; exit 1; }
wc -c gpurun_out/${T}_bench.json
python -c "
import json,sys; d=json.load(open('gpurun_out/${T}_bench.json'))
print('value', d['value'], 'frac', d['roofline']['frac'], 'tr', d['roofline'].get('traffic_ratio'), 'ok', d['checks_ok'])
print('target64', d.get('target64',{}).get('value'), d.get('target64',{}).get('ok'))
print({c:(r['value'], r['ok']) for c,r in d.get('configs',{}).items()})
print(d.get('cpu_baseline'))
"
echo "[$(date +%T)] rehearsal"
TAG=$T NS="${NS:-2}" bash tools/gpu_multirank_rehearsal.sh || exit 1
echo ALL_OK
