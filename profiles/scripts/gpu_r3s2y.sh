# A/B: MFMA wave priority in the attention kernels at D = 64 (FFK_ATTN_PRIO), GPT-3 medium (causal, attention-heavy).
set -o pipefail
bash tools/ab_env.sh FFK_ATTN_PRIO "--model gpt3-medium --steps 10 --warmup 3" ab_attn_prio_gpt_r3 0 1
