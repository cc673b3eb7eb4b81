# Round-4 checkpoint on one GPU: kernel A/B (optional), GPU tests, smoke, the
# default bench (C2 + stats roofline + target64 + C3/C4/C5 sub-records + PMC +
# CPU baseline), its rocprofv3 kernel trace, and the bench's N-rank launcher
# rehearsed on one GPU (2 ranks over gloo) plus its refusal without the knobs.
#   TAG=r04d AB="tools/ab_libs/x.so ..." AB_OPS=c5_k2v_runs bash tools/gpu_r04_checkpoint.sh
set -o pipefail
export TMPDIR=/tmp
T=${TAG:-r04d}
if [ -n "$AB" ]; then
  NAME=${T}_ab OPS=${AB_OPS:-c5_k2v_runs} ROUNDS=${AB_ROUNDS:-7} LIMIT=400 bash tools/gpu_ab.sh $AB || { echo AB_FAIL; exit 1; }
fi
echo "[$(date +%T)] gpu tests"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_gpu_tests.log 2>&1 || { echo TESTS_FAIL; tail -30 gpurun_out/${T}_gpu_tests.log; exit 1; }
tail -2 gpurun_out/${T}_gpu_tests.log
echo "[$(date +%T)] smoke"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 gpurun_out/${T}_smoke.log; exit 1; }
echo "[$(date +%T)] bench (default run)"
timeout -k 10 900 python bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { echo BENCH_FAIL; tail -30 gpurun_out/${T}_bench.err; exit 1; }
echo "[$(date +%T)] bench under rocprofv3 --kernel-trace --stats"
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof -o run --output-format csv -- python bench.py --no-pmc --no-cpu-baseline --no-checks > gpurun_out/${T}_prof.json 2> gpurun_out/${T}_prof.err || { echo PROF_FAIL; tail -20 gpurun_out/${T}_prof.err; exit 1; }
echo "[$(date +%T)] launcher rehearsal: --gpus 2 on one GPU over gloo"
BOLT_AMD_BENCH_BACKEND=gloo BOLT_AMD_BENCH_DEVICE=0 timeout -k 10 600 python bench.py --gpus 2 --steps 3 --warmup 1 --no-configs > gpurun_out/${T}_n2_rehearsal.json 2> gpurun_out/${T}_n2_rehearsal.err || { echo REHEARSAL_FAIL; tail -30 gpurun_out/${T}_n2_rehearsal.err; exit 1; }
echo "[$(date +%T)] --gpus 2 without the knobs on one GPU (must exit non-zero)"
timeout -k 10 120 python bench.py --gpus 2 --steps 1 > gpurun_out/${T}_n2_refused.json 2> gpurun_out/${T}_n2_refused.err && { echo REFUSAL_MISSING; exit 1; }
echo "refused with rc $? (expected)"
echo ALL_OK
