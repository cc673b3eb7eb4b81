# bench.py's N>1 path rehearsed on one GPU: 2 ranks on cuda:0 over gloo (host-staged exchanges)
set -o pipefail
export TMPDIR=/tmp
export BOLT_AMD_BENCH_BACKEND=gloo BOLT_AMD_BENCH_DEVICE=0
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 > gpurun_out/bench_n2_rehearsal.json 2> gpurun_out/bench_n2_rehearsal.err || { echo FAIL; exit 1; }
echo ALL_OK
