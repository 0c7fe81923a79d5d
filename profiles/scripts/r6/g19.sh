#!/bin/bash
# round 6, call 19: environment values dropped after their last forward reader -- GPU tier + every bench model's memory
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6g19; mkdir -p $O
cd $R
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tier.txt 2>&1
rc=$?; tail -3 $O/tier.txt; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
for m in bert-large gpt3-medium resnet50 resnext50 inception-v3 dlrm; do
  timeout -k 10 300 python3 $R/bench.py --model $m --steps 10 --warmup 3 > $O/bench_$m.log 2>&1 || { tail -20 $O/bench_$m.log; exit 1; }
  tail -1 $O/bench_$m.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; m=c.get('memory'); print(c['model'], d['value'], d['ms_per_step'], m['planned_arena_gb'], m['measured_step_peak_gb'], m['plan_error_pct'], m.get('device_arena'))"
done
