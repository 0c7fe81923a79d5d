#!/bin/bash
# round 6, call 44: conv weight-gradient split-K degree tuned per shape -- conv tests, then ResNet-50 (512) A/B
# against the kernel heuristic (FF_CONV_WGRAD_TUNE=0), interleaved
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6g44; mkdir -p $O
cd $R
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_conv_gpu.py \
  tests/test_conv_grouped_gpu.py > $O/tests.txt 2>&1
rc=$?; tail -2 $O/tests.txt; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
for i in 1 2; do for t in 1 0; do
  FF_CONV_WGRAD_TUNE=$t timeout -k 10 300 python3 $R/bench.py --model resnet50 --steps 10 --warmup 3 > $O/rn_t${t}_$i.jsonl 2> $O/rn_t${t}_$i.err || { tail -5 $O/rn_t${t}_$i.err; exit 1; }
  tail -1 $O/rn_t${t}_$i.jsonl | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('tune=$t', d['value'], d['ms_per_step'])"
done; done
