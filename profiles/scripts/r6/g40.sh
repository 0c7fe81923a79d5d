#!/bin/bash
# round 6, call 40: BERT-large per-GPU batch 64 vs 128 on HEAD (same box, interleaved)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6g40; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for i in 1 2; do for b in 64 128; do
  timeout -k 10 300 python3 $R/bench.py --batch-per-gpu $b --steps 10 --warmup 3 > $O/b${b}_$i.jsonl 2> $O/b${b}_$i.err || { tail -5 $O/b${b}_$i.err; exit 1; }
  tail -1 $O/b${b}_$i.jsonl | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print($b, d['value'], d['ms_per_step'], c['memory']['measured_step_peak_gb'], c['memory']['plan_error_pct'])"
done; done
