# HBM bytes of the C2 reduction kernels (k_red_rows): one counter per pass
set -o pipefail
export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c -d gpurun_out/pmc_red_$c -o pmc --output-format csv -- python tools/reduce_only.py > gpurun_out/pmc_red_$c.log 2>&1 || { echo PMC_FAIL $c; exit 1; }
done
echo ALL_OK
