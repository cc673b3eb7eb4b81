# bench.py's N>1 path rehearsed on one GPU: 2 ranks on cuda:0 over gloo
# (host-staged exchanges), the default C2 run and C1 -- the code path of the
# driver's scaling run, not a measurement of it
set -o pipefail
export TMPDIR=/tmp
export BOLT_AMD_BENCH_BACKEND=gloo BOLT_AMD_BENCH_DEVICE=0
T=${TAG:-r02}
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 > gpurun_out/bench_n2_rehearsal_$T.json 2> gpurun_out/bench_n2_rehearsal_$T.err || { echo FAIL; tail -20 gpurun_out/bench_n2_rehearsal_$T.err; exit 1; }
cat gpurun_out/bench_n2_rehearsal_$T.json
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 2 --steps 3 --warmup 1 --config C1 > gpurun_out/bench_n2_rehearsal_${T}_c1.json 2> gpurun_out/bench_n2_rehearsal_${T}_c1.err || { echo FAIL_C1; tail -20 gpurun_out/bench_n2_rehearsal_${T}_c1.err; exit 1; }
cat gpurun_out/bench_n2_rehearsal_${T}_c1.json
echo ALL_OK
