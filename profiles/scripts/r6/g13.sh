#!/bin/bash
# round 6, call 13: arena on one stream (eager, warm-up, capture): tests, then BERT-large phases
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6g13; mkdir -p $O
cd $R
export PYTHONPATH=$R FF_MEM_PHASES=1
FF_ARENA_TEST=1 timeout -k 10 300 python3 -u -X faulthandler -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_arena_gpu.py > $O/tests.txt 2>&1
rc=$?; tail -4 $O/tests.txt; [ $rc -eq 0 ] || exit $rc
FF_ARENA=1 timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 > $O/arena.txt 2>&1
rc=$?; grep "\[mem\]\|^{" $O/arena.txt; exit $rc
