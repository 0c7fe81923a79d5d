#!/bin/bash
# round 6, call 14: every bench model with the device arena on (default at N=1)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6g14; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for m in bert-large gpt3-medium resnet50 resnext50 inception-v3 dlrm; do
  timeout -k 10 300 python3 $R/bench.py --model $m --steps 10 --warmup 3 > $O/bench_$m.log 2>&1 || { tail -20 $O/bench_$m.log; exit 1; }
  tail -1 $O/bench_$m.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print(c['model'], d['value'], d['ms_per_step'], c.get('memory'))"
done
