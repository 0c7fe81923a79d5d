# round 5, call 20: rocprofv3 counters of the implicit-GEMM conv kernels (fwd / dgrad / wgrad)
# at the ResNet-50 layer-3 3x3 shape (14x14, 256 -> 256, batch 256)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5g20; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
    SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE --output-format csv -d $O/p1 -o c1 -- \
    python3 $R/tools/conv_pmc_one.py > $O/p1.log 2>&1 || { tail -20 $O/p1.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_WAIT_INST_LDS \
    SQ_INSTS_VMEM_RD SQ_INSTS_SALU TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE --output-format csv -d $O/p2 -o c2 -- \
    python3 $R/tools/conv_pmc_one.py > $O/p2.log 2>&1 || { tail -20 $O/p2.log; exit 1; }
for p in p1 p2; do CSV=$(find $O/$p -name "*counter_collection.csv" | head -n 1); python3 $R/tools/pmc_summary.py $CSV --raw > $O/$p.txt 2>&1; head -60 $O/$p.txt; done
