set -o pipefail
export TMPDIR=/tmp
for r in 1 2; do
  for v in p0 p1; do
    BOLT_AMD_LIB=$PWD/tools/ab_$v.so timeout -k 10 300 python tools/chunk_bench.py > gpurun_out/recmap_${v}_$r.log 2>&1 || { echo FAIL; exit 1; }
  done
done
echo ALL_OK
