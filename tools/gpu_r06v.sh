# Round 6, call v: the default bench with torch's caching allocator on plain
# hipMalloc segments (A) and on expandable segments (B: hipMemCreate /
# hipMemMap, PYTORCH_HIP_ALLOC_CONF=expandable_segments:True), A B A B in
# fresh processes on one box; PMC, CPU baseline and checks off.
set -o pipefail
export TMPDIR=/tmp
T=${TAG:-r06v}
mkdir -p gpurun_out
run() {
  timeout -k 10 420 python -u bench.py --no-cpu-baseline --no-pmc --no-checks --no-rocprof --detail gpurun_out/${T}_$1.detail.json > gpurun_out/${T}_$1.out 2> gpurun_out/${T}_$1.err || { echo RUN_FAIL $1; tail -20 gpurun_out/${T}_$1.err; exit 1; }
}
run A1
PYTORCH_HIP_ALLOC_CONF=expandable_segments:True run B1
run A2
PYTORCH_HIP_ALLOC_CONF=expandable_segments:True run B2
grep -i "expandable" gpurun_out/${T}_B1.err | head -3
python - <<'PY'
import json, os
T = os.environ.get("TAG", "r06v")
for k in ("A1", "B1", "A2", "B2"):
    d = json.loads(open("gpurun_out/%s_%s.out" % (T, k)).read().strip().splitlines()[-1])
    row = {"C2": d["value"], "C2.swap": d["ops"]["swap"]["ms"], "t64": d["target64"]["value"]}
    for c in ("C1", "C3", "C4", "C5"):
        row[c] = d["configs"][c]["value"]
    row.update({"C5." + n: o["ms"] for n, o in d["configs"]["C5"]["ops"].items()})
    print(k, json.dumps(row))
PY
echo ALL_OK
