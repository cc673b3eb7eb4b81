# HBM traffic of every kernel of a config's bench step: FETCH_SIZE and
# WRITE_SIZE in separate rocprofv3 --pmc passes (the MI355X guide's recipe;
# FETCH_SIZE doubled on gfx950), summarised per kernel by tools/pmc_kernels.py.
#   TAG=r03zk CONFIGS="C4 C5" bash tools/gpu_pmc_steps.sh
set -o pipefail
export TMPDIR=/tmp
T=${TAG:-r03zk}
for c in ${CONFIGS:-C4 C5}; do
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 300 rocprofv3 --pmc $ctr --kernel-trace -d gpurun_out/${T}_${c}_$ctr -o pmc --output-format csv -- python bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline --no-pmc > gpurun_out/${T}_${c}_$ctr.log 2>&1 || { echo PMC_FAIL $c $ctr; tail -5 gpurun_out/${T}_${c}_$ctr.log; exit 1; }
  done
  python tools/pmc_kernels.py gpurun_out/${T}_${c}_FETCH_SIZE gpurun_out/${T}_${c}_WRITE_SIZE > gpurun_out/${T}_${c}_traffic.txt && cat gpurun_out/${T}_${c}_traffic.txt
done
echo ALL_OK
