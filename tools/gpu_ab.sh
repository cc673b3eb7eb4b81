# Interleaved A/B of libbolt_mi355x builds in one process (tools/ab_bench.py),
# every output byte-compared between the variants (--check).
#   NAME=rot OPS=c2_swap,c5_T ROUNDS=7 bash tools/gpu_ab.sh tools/ab_libs/rot1.so [more.so]
# The in-tree library is always variant A.  Build variants on the CPU first:
#   make -C bolt_amd/csrc OUT=$PWD/tools/ab_libs/rot1.so BUILD=/tmp/brot EXTRA=-DBM_TR_ROT=1
set -o pipefail
export TMPDIR=/tmp
NAME=${NAME:-ab}
OPS=${OPS:-c2_swap,c5_T,c5_perm,c3_T,c3_swap}
ROUNDS=${ROUNDS:-7}
timeout -k 10 ${LIMIT:-700} python tools/ab_bench.py bolt_amd/libbolt_mi355x.so "$@" --ops $OPS --rounds $ROUNDS --placements ${PLACEMENTS:-1} --check > gpurun_out/ab_$NAME.log 2>&1 || { echo AB_FAIL; tail -20 gpurun_out/ab_$NAME.log; exit 1; }
cat gpurun_out/ab_$NAME.log
