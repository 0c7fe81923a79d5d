#!/bin/bash
# round 6, call 8: backward hand-offs released + autotune split-K slabs trimmed:
# GPU tier, memory audits, benches with the plan-vs-step-peak record
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6g08; mkdir -p $O
cd $R
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/gpu_tier.txt 2>&1
rc=$?
tail -4 $O/gpu_tier.txt
[ $rc -le 1 ] || exit $rc
for m in gpt bert-large resnet50; do
  PYTHONPATH=$R timeout -k 10 300 python3 $R/tools/mem_audit.py $m > $O/mem_$m.jsonl 2>&1 || { tail -20 $O/mem_$m.jsonl; exit 1; }
  head -1 $O/mem_$m.jsonl
done
cd /tmp && export TMPDIR=/tmp
for m in bert-large resnet50 gpt3-medium; do
  timeout -k 10 400 python3 $R/bench.py --model $m --steps 10 --warmup 3 > $O/bench_$m.log 2>&1 || { tail -20 $O/bench_$m.log; exit 1; }
  tail -1 $O/bench_$m.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['config']['model'], d['value'], d['config']['memory'])"
done
