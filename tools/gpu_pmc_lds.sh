# LDS counters of the transposes (u16 / u8 packed vs f32), one --pmc pass each.
set -o pipefail
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVES -d gpurun_out/pmc_lds1 -o run --output-format csv -- python tools/ab_bench.py bolt_amd/libbolt_mi355x.so --ops u16_T,u8_T,c2_swap --rounds 1 --reps 1 > gpurun_out/pmc_lds1.log 2>&1 || { echo PMC1_FAIL; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_VMEM_RD -d gpurun_out/pmc_lds2 -o run --output-format csv -- python tools/ab_bench.py bolt_amd/libbolt_mi355x.so --ops u16_T,u8_T,c2_swap --rounds 1 --reps 1 > gpurun_out/pmc_lds2.log 2>&1 || { echo PMC2_FAIL; exit 1; }
echo ALL_OK
