#!/bin/bash
# round 6, call 29: second bench run in one process -- one device without a process group, and RCCL at world 1
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6g29; mkdir -p $O
cd $R
WORLD_SIZE=1 RANK=0 ORDER=dp,dp FF_STEP_TIMES=1 timeout -k 10 300 python3 tools/diag/two_runs.py > $O/w1.out 2> $O/w1.err || { tail -30 $O/w1.err; exit 1; }
grep "^run" $O/w1.err
WORLD_SIZE=1 RANK=0 FF_DIST_WORLD1=1 ORDER=dp,dp FF_STEP_TIMES=1 timeout -k 10 300 python3 tools/diag/two_runs.py > $O/rccl1.out 2> $O/rccl1.err || { tail -30 $O/rccl1.err; exit 1; }
grep "^run\|\[step\]" $O/rccl1.err
