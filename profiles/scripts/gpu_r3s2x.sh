# A/B of the column-sum grid (FFK_COLSUM_BLOCKS 1024 default vs 2048) on batch-64 BERT-large.
set -o pipefail
bash tools/ab_env.sh FFK_COLSUM_BLOCKS "--steps 10 --warmup 3" ab_colsum_blocks_b64 1024 2048
