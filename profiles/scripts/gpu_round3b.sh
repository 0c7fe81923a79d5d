# gemmq sync ablation + PMC counters on two shapes (results under gpurun_out/)
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
timeout -k 10 300 python -u tools/gemm_ablate.py > gpurun_out/gemm_ablate.jsonl 2> gpurun_out/gemm_ablate.err && \
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VALU_MFMA_MOPS_BF16 GRBM_GUI_ACTIVE -d gpurun_out/pmc/q_dx -o q_dx -- python3 tools/gemmp_one.py 16384 1024 4096 0 1 1 > gpurun_out/pmc_q_dx.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VALU_MFMA_MOPS_BF16 GRBM_GUI_ACTIVE -d gpurun_out/pmc/q_qkv -o q_qkv -- python3 tools/gemmp_one.py 16384 3072 1024 0 0 1 > gpurun_out/pmc_q_qkv.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM SQ_INSTS_SALU SQ_INSTS_VALU SQ_WAVES SQ_INSTS_MFMA GRBM_GUI_ACTIVE -d gpurun_out/pmc/q_dx2 -o q_dx2 -- python3 tools/gemmp_one.py 16384 1024 4096 0 1 1 > gpurun_out/pmc_q_dx2.log 2>&1
