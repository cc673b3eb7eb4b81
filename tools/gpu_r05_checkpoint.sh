# Round-5 checkpoint on one GPU: GPU tests, smoke, optional interleaved A/B of
# library builds, the default bench, the same bench under rocprofv3
# --kernel-trace --stats, and the N-rank rehearsal (rank 0 under rocprofv3).
#   TAG=r05b AB="tools/ab_libs/r05_step1.so" AB_OPS=c2_swap,... bash tools/gpu_r05_checkpoint.sh
# SKIP="bench prof rehearsal" skips steps.
set -o pipefail
export TMPDIR=/tmp
T=${TAG:-r05b}
mkdir -p gpurun_out
skip() { case " $SKIP " in *" $1 "*) return 0;; esac; return 1; }
echo "[$(date +%T)] gpu tests"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_gpu_tests.log 2>&1 || { echo TESTS_FAIL; tail -30 gpurun_out/${T}_gpu_tests.log; exit 1; }
tail -1 gpurun_out/${T}_gpu_tests.log
echo "[$(date +%T)] smoke"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 gpurun_out/${T}_smoke.log; exit 1; }
tail -1 gpurun_out/${T}_smoke.log
if [ -n "$AB" ]; then
  echo "[$(date +%T)] A/B"
  NAME=${T} OPS=${AB_OPS:-c2_swap,c3_full,c3T_full,c4_full,c5_T,c5_perm} ROUNDS=${AB_ROUNDS:-7} LIMIT=500 bash tools/gpu_ab.sh $AB || { echo AB_FAIL; exit 1; }
fi
if ! skip bench; then
  echo "[$(date +%T)] bench (default run)"
  timeout -k 10 900 python bench.py --detail gpurun_out/${T}_bench_detail.json > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { echo BENCH_FAIL; tail -30 gpurun_out/${T}_bench.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/${T}_bench.json'))
print('value', d['value'], 'frac', d['roofline']['frac'], 'tr', d['roofline'].get('traffic_ratio'), 'ok', d['checks_ok'], 'chars', len(open('gpurun_out/${T}_bench.json').read()))
print('target64', d.get('target64',{}).get('value'), d.get('target64',{}).get('ok'))
print({c:(r['value'], r['ok']) for c,r in d.get('configs',{}).items()})"
fi
if ! skip prof; then
  echo "[$(date +%T)] bench under rocprofv3 --kernel-trace --stats"
  timeout -k 10 900 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof -o run --output-format csv -- python bench.py --no-pmc --no-cpu-baseline --no-checks --detail gpurun_out/${T}_prof_detail.json > gpurun_out/${T}_prof.json 2> gpurun_out/${T}_prof.err || { echo PROF_FAIL; tail -20 gpurun_out/${T}_prof.err; exit 1; }
fi
if ! skip rehearsal; then
  echo "[$(date +%T)] rehearsal"
  TAG=$T NS="${NS:-2}" bash tools/gpu_multirank_rehearsal.sh || exit 1
fi
echo ALL_OK
