#!/bin/bash
# round 6, call 46: BERT-large autotune report at 128 sequences / GPU (which GEMM signatures go to the library, margins)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6g46; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
FF_GEMM_REPORT=1 timeout -k 10 300 python3 $R/bench.py --steps 5 --warmup 2 > $O/bench.jsonl 2> $O/bench.err
rc=$?; grep "^a\[\|^dact" $O/bench.err > $O/autotune.txt; cat $O/autotune.txt | cut -c1-220; exit $rc
