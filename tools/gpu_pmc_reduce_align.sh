# k_red_rows over-fetch attribution: FETCH_SIZE / WRITE_SIZE passes over
# tools/reduce_align.py (8000-B vs 8192-B rows), one counter per pass.
set -o pipefail
export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c -d gpurun_out/pmc_align_$c -o pmc --output-format csv -- python tools/reduce_align.py > gpurun_out/pmc_align_$c.log 2>&1 || { echo PMC_FAIL $c; exit 1; }
done
echo ALL_OK
