# Round 6, call d: checkpoint (GPU suite, smoke, default bench) after the
# unit-axis / padded-egress / multi-rank-pitch changes, then the rows
# reduction's read requests by size (the 1.018x FETCH_SIZE of padded C2 rows,
# VERDICT r05 next #6) against a plain copy of the same bytes.
set -o pipefail
export TMPDIR=/tmp
T=${TAG:-r06d}
TAG=$T SKIP="${SKIP:-prof rehearsal}" bash tools/gpu_r05_checkpoint.sh || exit 1
L=bolt_amd/libbolt_mi355x.so
OPS=c2_mean_prow,c2_sum_prow,c2_mean_rows,c2_sum_rows
i=0
for grp in "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum" \
           "TCP_TCC_READ_REQ_sum TCC_REQ_sum TCC_HIT_sum TCC_MISS_sum" \
           "FETCH_SIZE"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $grp --kernel-trace -d gpurun_out/${T}_rq_$i -o pmc --output-format csv -- python tools/ab_bench.py $L --ops c2_copy,$OPS --rounds 1 --reps 1 > gpurun_out/${T}_rq_$i.log 2>&1 || { echo RQ_FAIL $i; tail -5 gpurun_out/${T}_rq_$i.log; break; }
done
python tools/ab_pmc_table.py --ops $OPS --libs lib --kernel k_red_rows gpurun_out/${T}_rq_[123] > gpurun_out/${T}_rq_table.md
python tools/ab_pmc_table.py --ops c2_copy --libs lib --kernel k_rowcopy gpurun_out/${T}_rq_[123] >> gpurun_out/${T}_rq_table.md
cat gpurun_out/${T}_rq_table.md
echo ALL_OK
