#!/bin/bash
# round 6, call 43: ResNet-50 (default batch 512) kernel trace on HEAD -- where the BN passes stand
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6g43; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_rn50 -o rn -- \
    python3 $R/bench.py --model resnet50 --steps 10 --warmup 3 > $O/prof_rn50.log 2>&1 || { tail -20 $O/prof_rn50.log; exit 1; }
DB=$(find $O/prof_rn50 -name "rn_results.db" | head -n 1)
[ -n "$DB" ] && python3 $R/tools/prof_summary.py $DB --steps 5 --top 40 > $O/rn50_kernels.txt
head -45 $O/rn50_kernels.txt
