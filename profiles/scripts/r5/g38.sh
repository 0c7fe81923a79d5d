#!/bin/bash
# round 5, call 38: HBM bytes of the ResNet-50 BN passes (FETCH_SIZE / WRITE_SIZE, one pass each)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5g38; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/f -o run -- python3 $R/bench.py --model resnet50 --steps 2 --warmup 1 > $O/f.log 2>&1 || { tail -20 $O/f.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/w -o run -- python3 $R/bench.py --model resnet50 --steps 2 --warmup 1 > $O/w.log 2>&1 || { tail -20 $O/w.log; exit 1; }
python3 $R/tools/rocpd_pmc.py $(find $O/f -name "*.db" | head -n 1) > $O/fetch.txt 2>&1
python3 $R/tools/rocpd_pmc.py $(find $O/w -name "*.db" | head -n 1) > $O/write.txt 2>&1
rm -rf $O/f $O/w
