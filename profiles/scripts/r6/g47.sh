#!/bin/bash
# round 6, call 47: every bench model at its round-6 default batch on HEAD (20 timed steps)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6g47; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for m in bert-large gpt3-medium resnet50 resnext50 inception-v3 dlrm; do
  timeout -k 10 300 python3 $R/bench.py --model $m --steps 20 --warmup 5 > $O/bench_$m.jsonl 2> $O/bench_$m.err || { tail -20 $O/bench_$m.err; exit 1; }
  tail -1 $O/bench_$m.jsonl | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; m=c.get('memory'); print(c['model'], c['global_batch'], d['value'], d['ms_per_step'], m['planned_arena_gb'], m['measured_step_peak_gb'], m['plan_error_pct'], (m.get('device_arena') or {}).get('overflow_segments'))"
done
