# Round 6, call o: the C5 pack against a plain copy on the same buffers
# (tools/c5_place_bench.py) -- the C5 config alone, then the default run
# (checks on; PMC passes on in the last run, as the driver runs it).
set -o pipefail
export TMPDIR=/tmp
T=${TAG:-r06o}
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/c5_place_bench.py --config C5 --steps 3 --warmup 1 --no-cpu-baseline --no-pmc --no-sweeps --no-rocprof > gpurun_out/${T}_c5.out 2> gpurun_out/${T}_c5.err || { echo C5_FAIL; tail -20 gpurun_out/${T}_c5.err; exit 1; }
grep GATHER gpurun_out/${T}_c5.err | tail -4
timeout -k 10 700 python -u tools/c5_place_bench.py --no-cpu-baseline --no-pmc --no-rocprof > gpurun_out/${T}_full.out 2> gpurun_out/${T}_full.err || { echo FULL_FAIL; tail -20 gpurun_out/${T}_full.err; exit 1; }
grep GATHER gpurun_out/${T}_full.err | tail -4
[ -n "$WITH_PMC" ] && { timeout -k 10 700 python -u tools/c5_place_bench.py --no-cpu-baseline --no-rocprof > gpurun_out/${T}_pmc.out 2> gpurun_out/${T}_pmc.err || { echo PMC_FAIL; tail -20 gpurun_out/${T}_pmc.err; exit 1; }; }
[ -n "$WITH_PMC" ] && grep GATHER gpurun_out/${T}_pmc.err | tail -4
echo ALL_OK
