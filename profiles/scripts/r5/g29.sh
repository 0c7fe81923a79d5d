# round 5, call 29: counters of the ping-pong A B^T kernel (variant 11) vs hipBLASLt and the
# one-wave kernel (variant 6) on the BERT dX FFN1 shape (32768 x 4096 x 1024, A B^T)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5g29; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_BUSY_CYCLES \
    SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d $O/p1 -o g1 -- \
    python3 $R/tools/gemm_pmc_one.py 32768 4096 1024 0 1 6 11 > $O/p1.log 2>&1 || { tail -20 $O/p1.log; exit 1; }
CSV=$(find $O/p1 -name "*counter_collection.csv" | head -n 1)
python3 $R/tools/pmc_summary.py $CSV > $O/pmc.txt 2>&1; head -50 $O/pmc.txt
