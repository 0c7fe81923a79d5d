#!/bin/bash
# round 6, call 12: memory after each set-up phase, torch allocator vs device arena (BERT-large)
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6g12; mkdir -p $O
cd $R
export PYTHONPATH=$R FF_MEM_PHASES=1
timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 2 > $O/torch.txt 2>&1
rc=$?; grep "\[mem\]" $O/torch.txt; [ $rc -eq 0 ] || exit $rc
FF_ARENA=1 timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 2 > $O/arena.txt 2>&1
rc=$?; grep "\[mem\]" $O/arena.txt; exit $rc
