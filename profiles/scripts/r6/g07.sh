#!/bin/bash
# round 6, call 7: where the persistent base of the GPT / BERT / ResNet steps sits (allocation sites)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6g07; mkdir -p $O
cd $R
for m in gpt bert-large resnet50; do
  PYTHONPATH=$R timeout -k 10 300 python3 $R/tools/mem_audit.py $m --trace > $O/mem_$m.jsonl 2>&1 || { tail -20 $O/mem_$m.jsonl; exit 1; }
  grep base_site $O/mem_$m.jsonl | head -12
done
