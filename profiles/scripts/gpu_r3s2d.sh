# PMC counters of the attention kernels (tools/attn_time.py, both shapes), one pass per counter group.
set -o pipefail
mkdir -p gpurun_out/pmc_attn
export TMPDIR=/tmp
export FFK_ATTN_BWD_PF=1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE -d gpurun_out/pmc_attn/p1 -o p1 --output-format csv -- python3 tools/attn_time.py 5 > gpurun_out/pmc_attn/p1.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_WAVES -d gpurun_out/pmc_attn/p2 -o p2 --output-format csv -- python3 tools/attn_time.py 5 > gpurun_out/pmc_attn/p2.log 2>&1
