#!/bin/bash
# round 6, call 15: arena answers "no room" once so torch's cache releases before overflow
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6g15; mkdir -p $O
cd $R
timeout -k 10 300 python3 -u -X faulthandler -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_arena_gpu.py > $O/tests.txt 2>&1
rc=$?; tail -4 $O/tests.txt; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
for m in gpt3-medium resnet50 bert-large; do
  timeout -k 10 300 python3 $R/bench.py --model $m --steps 10 --warmup 3 > $O/bench_$m.log 2>&1 || { tail -20 $O/bench_$m.log; exit 1; }
  tail -1 $O/bench_$m.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print(c['model'], d['value'], d['ms_per_step'], c.get('memory'))"
done
