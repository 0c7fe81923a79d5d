#!/bin/bash
# round 6, call 30: thread-local capture mode -- RCCL world 1, two bench runs in one process (segmented capture with
# the RCCL watchdog alive), then the segmented-graph GPU tests
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6g30; mkdir -p $O
cd $R
WORLD_SIZE=1 RANK=0 FF_DIST_WORLD1=1 ORDER=dp,dp FF_STEP_TIMES=1 timeout -k 10 300 python3 tools/diag/two_runs.py > $O/rccl1.out 2> $O/rccl1.err || { grep -v "^frame" $O/rccl1.err | tail -20; exit 1; }
grep "^run\|\[step\]" $O/rccl1.err
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_segmented_graph_gpu.py tests/test_rccl_gpu.py tests/test_pipeline_graph_gpu.py > $O/tests.txt 2>&1
rc=$?; tail -3 $O/tests.txt; exit $rc
