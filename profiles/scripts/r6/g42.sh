#!/bin/bash
# round 6, call 42: GPT-3 medium 16 vs 32 sequences / GPU and ResNet-50 256 vs 512 images / GPU (same box, interleaved)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6g42; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for cfg in "gpt3-medium 16" "gpt3-medium 32" "resnet50 256" "resnet50 512" "gpt3-medium 16" "gpt3-medium 32" "resnet50 256" "resnet50 512"; do
  set -- $cfg
  timeout -k 10 300 python3 $R/bench.py --model $1 --batch-per-gpu $2 --steps 10 --warmup 3 > $O/$1_$2.jsonl 2> $O/$1_$2.err || { tail -5 $O/$1_$2.err; exit 1; }
  tail -1 $O/$1_$2.jsonl | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print('$1', $2, d['value'], d['ms_per_step'], c['memory']['measured_step_peak_gb'], c['memory']['plan_error_pct'])"
done
