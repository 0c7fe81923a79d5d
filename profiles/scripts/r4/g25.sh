# round 4, call 25: counters of gemmt_kk_kernel on the NT input gradient (BERT FFN1 dX) next to hipBLASLt
# BERT FFN1 shape, split 4; NN forward FFN1 shape) next to hipBLASLt
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4g25; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
C1="GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY"
C2="GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_VALU SQ_INSTS_MFMA"
for SH in "32768 1024 4096 0 1 6:1"; do
  TAG=$(echo $SH | cut -d' ' -f1-5 | tr ' ' '_')
  for P in 1 2; do
    eval CC=\$C$P
    timeout -s KILL 90 rocprofv3 --pmc $CC --output-format csv -d $O/pmc_g_${TAG}_$P -o g -- \
        python3 $R/tools/gemm_pmc_one.py $SH > $O/pmc_g_${TAG}_$P.log 2>&1 \
        || { tail -5 $O/pmc_g_${TAG}_$P.log; exit 1; }
    CSV=$(find $O/pmc_g_${TAG}_$P -name "*counter_collection.csv" | head -n 1)
    python3 $R/tools/pmc_summary.py $CSV --raw > $O/pmc_g_${TAG}_$P.txt
    rm -rf $O/pmc_g_${TAG}_$P
  done
done
cat $O/*.txt
