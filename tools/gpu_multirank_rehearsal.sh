# bench.py's N-rank path with every sub-record, rehearsed on ONE GPU: N ranks
# share cuda:0, exchanges staged through the host over gloo (RCCL refuses two
# ranks on one GPU) -- the code path of the driver's scaling run (events,
# checks of every op, strong-scaled sub-records, rank 0 under rocprofv3
# --kernel-trace with the marked pass), at reduced shapes; not a measurement.
#   TAG=r05g NS="2 4" [LAUNCH=torchrun] bash tools/gpu_multirank_rehearsal.sh
set -o pipefail
export TMPDIR=/tmp
T=${TAG:-r05g}
SHAPES=${SHAPES:-'{"C1":[100,64,64],"C2":[200,512,512],"C3":[256,256,256,32],"C4":[800,1024,1024],"C5":[16,64,64,64,64]}'}
for n in ${NS:-2 4}; do
  echo "[$(date +%T)] $n ranks"
  if [ "$LAUNCH" = torchrun ]; then
    # the driver's launch: torch.distributed.run starts the ranks (bench.py's rank 0 then re-runs
    # itself under rocprofv3 before touching the GPU)
    L="python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29500 + n))"
  else
    L="python"
  fi
  BOLT_AMD_BENCH_BACKEND=gloo BOLT_AMD_BENCH_DEVICE=0 timeout -k 10 600 $L bench.py --gpus $n --steps 3 --warmup 1 --shapes "$SHAPES" --detail gpurun_out/${T}_n${n}_detail.json > gpurun_out/${T}_n${n}_rehearsal.json 2> gpurun_out/${T}_n${n}_rehearsal.err || { echo REHEARSAL_FAIL $n; tail -30 gpurun_out/${T}_n${n}_rehearsal.err; exit 1; }
  python - gpurun_out/${T}_n${n}_rehearsal.json <<'PY'
import json, sys
d = json.loads([ln for ln in open(sys.argv[1]).read().splitlines() if ln.startswith("{")][-1])
print("n_gpus", d["n_gpus"], "exchange_check", d.get("exchange_check"), "launcher", d.get("launcher"), "chars", len(json.dumps(d, separators=(",", ":"))))
recs = [("C2", d)] + list(d.get("configs", {}).items())
bad = [(c, k, o.get("ck")) for c, r in recs for k, o in r["ops"].items()
       if not (o.get("ck") == "exact" or str(o.get("ck")).startswith("ok "))]
print("checks", {c: r.get("ok", r.get("checks_ok")) for c, r in recs}, "bad", bad)
rp = d.get("rocprof") or {}
print("rocprof", rp.get("error"), rp.get("stats"))
for k, v in sorted((rp.get("ops") or {}).items()):
    print("  ", k, v)
ok = not bad and d["n_gpus"] >= 2 and not rp.get("error") and (rp.get("ops") or {}).get("C2.swap", {}).get("lib", 0) > 0
sys.exit(0 if ok else 1)
PY
  [ $? -eq 0 ] || { echo CHECKS_FAIL $n; exit 1; }
done
echo ALL_OK
