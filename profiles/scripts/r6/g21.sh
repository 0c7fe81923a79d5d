#!/bin/bash
# round 6, call 21: one-device graph replay through the native replayer; arena / graph tests, smoke, BERT bench
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6g21; mkdir -p $O
cd $R
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_arena_gpu.py tests/test_segmented_graph_gpu.py tests/test_pipeline_graph_gpu.py tests/test_executor_gpu.py > $O/tests.txt 2>&1
rc=$?; tail -3 $O/tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1
rc=$?; tail -2 $O/smoke.txt; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python3 $R/bench.py > $O/bench.log 2>&1
rc=$?; tail -1 $O/bench.log | cut -c1-400; exit $rc
