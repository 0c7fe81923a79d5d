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
# weight-gradient (TN, both operands K-outer) GEMM at the BERT FFN1 shape vs
# the NT input gradient: hipBLASLt, gemmt variant 6 (both operands by LDS-DMA)
# and 3 (register staging), split-K 4 — MFMA busy, wait / LDS counters, L2 hits
C1="GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY"
C2="GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_VALU SQ_INSTS_MFMA"
for SH in "1024 4096 32768 1 0 6:4 3:4" "32768 1024 4096 0 1 6:1 4:1"; do
  TAG=$(echo $SH | cut -d' ' -f1-5 | tr ' ' '_')
  for P in 1 2; do
    eval CC=\$C$P
    timeout -s KILL 90 rocprofv3 --pmc $CC --output-format csv -d $R/gpurun_out/r4g08/pmc_g_${TAG}_$P -o g -- \
        python3 $R/tools/gemm_pmc_one.py $SH > $R/gpurun_out/r4g08/pmc_g_${TAG}_$P.log 2>&1 \
        || { tail -5 $R/gpurun_out/r4g08/pmc_g_${TAG}_$P.log; exit 1; }
    CSV=$(find $R/gpurun_out/r4g08/pmc_g_${TAG}_$P -name "*counter_collection.csv" | head -n 1)
    python3 $R/tools/pmc_summary.py $CSV --raw > $R/gpurun_out/r4g08/pmc_g_${TAG}_$P.txt
  done
done
echo gemm pmc done
cd $R && timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r4g08/bench_bert.json 2> gpurun_out/r4g08/bench_bert.err || exit 1
tail -1 gpurun_out/r4g08/bench_bert.json | cut -c1-200
