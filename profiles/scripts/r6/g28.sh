#!/bin/bash
# round 6, call 28: is any second bench run in one process slow (gloo ranks on one GPU), or only after a searched run?
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6g28; mkdir -p $O
cd $R
for ORD in dp,dp search,search; do
  ORDER=$ORD FF_BENCH_REHEARSAL=1 FF_DIST_BACKEND=gloo FF_STEP_TIMES=1 timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 \
    --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29523 tools/diag/two_runs.py > $O/$ORD.out 2> $O/$ORD.err \
    || { tail -30 $O/$ORD.err; exit 1; }
  grep "^run\|\[step\]" $O/$ORD.err | head -20
done
