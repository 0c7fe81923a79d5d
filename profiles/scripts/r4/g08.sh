# round 4, call 8: per-kernel time of the BERT-large bench step (kernel trace,
# last 5 optimizer steps) and one counter pass over the attention kernels
# (MFMA busy %, achieved bf16 TFLOP/s, LDS bank conflicts) at both bench shapes
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r4g08
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r4g08/prof_bert -o bert -- \
    python3 $R/bench.py --steps 5 --warmup 3 > $R/gpurun_out/r4g08/prof_bert.log 2>&1 || { tail -20 $R/gpurun_out/r4g08/prof_bert.log; exit 1; }
tail -1 $R/gpurun_out/r4g08/prof_bert.log | cut -c1-200
DB=$(ls $R/gpurun_out/r4g08/prof_bert/*/bert_results.db 2>/dev/null | head -n 1 || true)
[ -z "$DB" ] && DB=$(ls $R/gpurun_out/r4g08/prof_bert/bert_results.db 2>/dev/null || true)
[ -n "$DB" ] && python3 $R/tools/prof_summary.py $DB --steps 5 --top 40 > $R/gpurun_out/r4g08/bert_kernels.txt
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 \
    SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_BUSY_CYCLES --output-format csv \
    -d $R/gpurun_out/r4g08/pmc_attn -o attn -- python3 $R/tools/attn_time.py --pmc-run \
    > $R/gpurun_out/r4g08/pmc_attn.log 2>&1 || { tail -20 $R/gpurun_out/r4g08/pmc_attn.log; exit 1; }
CSV=$(find $R/gpurun_out/r4g08/pmc_attn -name "*counter_collection.csv" | head -n 1)
python3 $R/tools/pmc_summary.py $CSV > $R/gpurun_out/r4g08/pmc_attn.txt
cat $R/gpurun_out/r4g08/pmc_attn.txt
