run() { timeout -k 10 200 env "$@" python bench.py --no-target64 --no-configs --no-pmc --no-cpu-baseline --no-checks 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(sys.argv[1], d['value'], d['ms_per_step'], d['roofline']['avg_ms'], d['stats_roofline']['mean']['avg_ms'])" "$*"; }
for i in 1 2 3; do
  run A=1 || exit 1
  run HSA_ENABLE_INTERRUPT=0 || exit 1
  run HIP_FORCE_DEV_KERNARG=1 || exit 1
  run HSA_ENABLE_INTERRUPT=0 HIP_FORCE_DEV_KERNARG=1 || exit 1
done
