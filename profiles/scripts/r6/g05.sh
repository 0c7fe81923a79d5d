#!/bin/bash
# round 6, call 5: segmented-graph / RCCL tests (stage-boundary plan), bench
# memory records (fusion-aware plan vs a steady-state step peak)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6g05; mkdir -p $O
cd $R
timeout -k 10 400 python3 -u -m pytest -q --timeout 120 --timeout-method thread tests/test_segmented_graph_gpu.py tests/test_rccl_gpu.py > $O/tests.txt 2>&1
rc=$?
tail -4 $O/tests.txt
[ $rc -le 1 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
for m in bert-large resnet50 gpt3-medium; do
  timeout -k 10 400 python3 $R/bench.py --model $m --steps 10 --warmup 3 > $O/bench_$m.log 2>&1 || { tail -20 $O/bench_$m.log; exit 1; }
  tail -1 $O/bench_$m.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['config']['model'], d['value'], d['config']['memory'])"
done
