#!/bin/bash
# round 6, call 11: arena tests after the init-order fix, then BERT-large with the arena on
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6g11; mkdir -p $O
cd $R
export PYTHONPATH=$R
FF_ARENA_TEST=1 timeout -k 10 300 python3 -u -X faulthandler -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_arena_gpu.py > $O/tests.txt 2>&1
rc=$?; echo "tests rc=$rc" >> $O/tests.txt; tail -5 $O/tests.txt
[ $rc -eq 0 ] || exit $rc
FF_ARENA=1 timeout -k 10 400 python3 -u bench.py --steps 20 --warmup 5 > $O/bench_arena.txt 2>&1
rc=$?; echo "bench rc=$rc" >> $O/bench_arena.txt; tail -3 $O/bench_arena.txt
