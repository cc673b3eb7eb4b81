# bench.py's N-rank path with every sub-record, rehearsed on ONE GPU: N ranks
# share cuda:0, exchanges staged through the host over gloo (RCCL refuses two
# ranks on one GPU) -- the code path of the driver's scaling run (events,
# checks, sub-records at world N), at reduced per-rank shapes; not a measurement.
#   TAG=r04g NS="2 4" bash tools/gpu_multirank_rehearsal.sh
set -o pipefail
export TMPDIR=/tmp
T=${TAG:-r04g}
SHAPES=${SHAPES:-'{"C1":[100,64,64],"C2":[200,512,512],"C3":[64,256,256,32],"C4":[200,1024,1024],"C5":[4,64,64,64,64]}'}
for n in ${NS:-2 4}; do
  echo "[$(date +%T)] $n ranks"
  BOLT_AMD_BENCH_BACKEND=gloo BOLT_AMD_BENCH_DEVICE=0 timeout -k 10 600 python bench.py --gpus $n --steps 3 --warmup 1 --shard-shapes "$SHAPES" > gpurun_out/${T}_n${n}_rehearsal.json 2> gpurun_out/${T}_n${n}_rehearsal.err || { echo REHEARSAL_FAIL $n; tail -30 gpurun_out/${T}_n${n}_rehearsal.err; exit 1; }
  python - gpurun_out/${T}_n${n}_rehearsal.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print("n_gpus", d["n_gpus"], "exchange_check", d["exchange_check"], "launcher", d.get("launcher"))
bad = [(c, k, v) for c, r in [("C2", d)] + list(d.get("configs", {}).items()) for k, v in (r.get("checks") or {}).items()
       if k != "all" and not (v == "bit-exact" or v.startswith("within"))]
print("configs", {c: r["checks"].get("all", "")[:20] for c, r in d.get("configs", {}).items()})
print("C4 var", d["configs"]["C4"]["checks"].get("var"))
sys.exit(1 if bad or d["n_gpus"] < 2 else 0)
PY
  [ $? -eq 0 ] || { echo CHECKS_FAIL $n; exit 1; }
done
echo ALL_OK
