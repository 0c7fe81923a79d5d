# Multi-rank rehearsal on ONE GPU: N ranks share cuda:0 over gloo (RCCL needs
# one GPU per rank; gloo exercises the same executor / bucketing / redistribution
# code with GPU tensors).  Usage: bash tools/rehearse_multi.sh [N] [model]
set -o pipefail
N=${1:-2}
MODEL=${2:-bert-large}
FF_BENCH_REHEARSAL=1 FF_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node "$N" \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --model "$MODEL" --gpus "$N" --steps 3 --warmup 1
