set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
C1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VALU_MFMA_MOPS_BF16 GRBM_GUI_ACTIVE"
C2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM SQ_INSTS_SALU SQ_INSTS_VALU SQ_WAVES SQ_INSTS_MFMA GRBM_GUI_ACTIVE"
C3="TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE SQ_INSTS_SMEM SQ_INST_CYCLES_VMEM SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL"
timeout -s KILL 90 rocprofv3 --pmc $C1 -d gpurun_out/pmc/c1 -o c1 -- python3 tools/gemm_pmc_one.py 16384 1024 4096 0 1 1 3 > gpurun_out/pmc_c1.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc $C2 -d gpurun_out/pmc/c2 -o c2 -- python3 tools/gemm_pmc_one.py 16384 1024 4096 0 1 1 3 > gpurun_out/pmc_c2.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc $C3 -d gpurun_out/pmc/c3 -o c3 -- python3 tools/gemm_pmc_one.py 16384 1024 4096 0 1 1 3 > gpurun_out/pmc_c3.log 2>&1
