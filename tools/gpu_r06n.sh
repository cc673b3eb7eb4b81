# Round 6, call n: is C5's chunk pack time (3.2-4.0 ms across bench runs)
# a property of the box, of the process, or of what ran before it?  The C5
# config alone in three fresh processes, then the default run's order
# (C2, target64, C1, C3, C4, C5) once, checks and PMC off.
set -o pipefail
export TMPDIR=/tmp
T=${TAG:-r06n}
mkdir -p gpurun_out
for i in 1 2 3; do
  timeout -k 10 240 python -u bench.py --config C5 --steps 5 --warmup 2 --no-cpu-baseline --no-pmc --no-checks --no-sweeps --no-rocprof --detail gpurun_out/${T}_c5_$i.json > gpurun_out/${T}_c5_$i.out 2> gpurun_out/${T}_c5_$i.err || { echo C5_FAIL $i; tail -20 gpurun_out/${T}_c5_$i.err; exit 1; }
done
timeout -k 10 600 python -u bench.py --no-cpu-baseline --no-pmc --no-checks --no-sweeps --no-rocprof --detail gpurun_out/${T}_full.json > gpurun_out/${T}_full.out 2> gpurun_out/${T}_full.err || { echo FULL_FAIL; tail -20 gpurun_out/${T}_full.err; exit 1; }
python - <<'PY'
import json, os
T = os.environ.get("TAG", "r06n")
for f in ["%s_c5_%d.out" % (T, i) for i in (1, 2, 3)] + ["%s_full.out" % T]:
    d = json.loads(open("gpurun_out/" + f).read().strip().splitlines()[-1])
    c = d["configs"]["C5"] if "configs" in d and "C5" in d["configs"] else d
    print(f, {k: v.get("ms") for k, v in c["ops"].items()})
PY
echo ALL_OK
