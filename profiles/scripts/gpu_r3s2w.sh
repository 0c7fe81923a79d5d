# 2-rank gloo rehearsal of GPT-3 medium on one GPU (pre-LN, causal attention) at the new default batch.
set -o pipefail
bash tools/rehearse_multi.sh 2 gpt3-medium > gpurun_out/rehearse2_gpt.log 2>&1
