#!/bin/bash
# round 5, call 40: BN reduction grid size (FFK_BN_RED_BLOCKS) A/B on ResNet-50, interleaved
set -o pipefail
O=gpurun_out/r5g40; mkdir -p $O
for b in 2048 1024 512 2048 1024 512; do
  FFK_BN_RED_BLOCKS=$b timeout -k 10 200 python bench.py --model resnet50 --steps 20 --warmup 5 >> $O/ab.jsonl 2>> $O/err.txt || exit 1
  echo "blocks=$b" >> $O/ab.jsonl
done
