#!/bin/bash
# round 5, call 43: BN apply-pass workgroup cap (FFK_BN_APPLY_BLOCKS) A/B on ResNet-50, interleaved
set -o pipefail
O=gpurun_out/r5g43; mkdir -p $O
for b in 8192 2048 4096 8192 2048 4096; do
  FFK_BN_APPLY_BLOCKS=$b timeout -k 10 200 python bench.py --model resnet50 --steps 20 --warmup 5 >> $O/ab.jsonl 2>> $O/err.txt || exit 1
  echo "blocks=$b" >> $O/ab.jsonl
done
