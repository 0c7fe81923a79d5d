#!/bin/bash
# round 6, call 10: where the MemPool + pluggable allocator path stops
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6g10; mkdir -p $O
cd $R
PYTHONPATH=$R timeout -k 10 120 python3 -u tools/arena_probe.py > $O/probe.txt 2>&1
echo "rc=$?" >> $O/probe.txt
grep -v "^  File\|^    " $O/probe.txt | head -30
