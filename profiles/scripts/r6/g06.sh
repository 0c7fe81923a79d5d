#!/bin/bash
# round 6, call 6: pipelined-step graph capture test, memory audits (GPT-3
# medium, ResNet-50, BERT-large) with the persistent base and the step peak
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6g06; mkdir -p $O
cd $R
timeout -k 10 300 python3 -u -m pytest -q --timeout 120 --timeout-method thread tests/test_pipeline_graph_gpu.py > $O/tests.txt 2>&1
rc=$?
tail -15 $O/tests.txt
[ $rc -le 1 ] || exit $rc
for m in gpt resnet50 bert-large; do
  PYTHONPATH=$R timeout -k 10 300 python3 $R/tools/mem_audit.py $m > $O/mem_$m.jsonl 2>&1 || { tail -20 $O/mem_$m.jsonl; exit 1; }
  head -12 $O/mem_$m.jsonl
done
