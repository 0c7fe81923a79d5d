#!/bin/bash
# round 6, call 9: the step's device arena (plan-sized, native allocator under a MemPool)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6g09; mkdir -p $O
cd $R
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_arena_gpu.py > $O/tests.txt 2>&1
rc=$?
tail -30 $O/tests.txt
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
for m in bert-large resnet50; do
  timeout -k 10 400 python3 $R/bench.py --model $m --steps 10 --warmup 3 > $O/bench_$m.log 2>&1 || { tail -20 $O/bench_$m.log; exit 1; }
  tail -1 $O/bench_$m.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['config']['model'], d['value'], d['config']['memory'])"
done
