#!/bin/bash
# round 6, call 17: GPT-3 medium with the split-K candidate bound + arena, then the whole GPU tier
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6g17; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python3 $R/bench.py --model gpt3-medium --steps 10 --warmup 3 > $O/bench_gpt.log 2>&1 || { tail -20 $O/bench_gpt.log; exit 1; }
tail -1 $O/bench_gpt.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print(c['model'], d['value'], d['ms_per_step'], c.get('memory'))"
cd $R
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tier.txt 2>&1
rc=$?; tail -5 $O/tier.txt; exit $rc
