#!/bin/bash
# dgrad BN sums only where the native dgrad is picked: A/B + kernel stats both ways
set -o pipefail
mkdir -p gpurun_out/r5g35
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 300 python bench.py --model resnet50 --steps 20 --warmup 5 > gpurun_out/r5g35/rn50_on.json 2> gpurun_out/r5g35/err.txt &&
FF_CONV_BN_BWD=0 timeout -k 10 300 python bench.py --model resnet50 --steps 20 --warmup 5 > gpurun_out/r5g35/rn50_off.json 2>> gpurun_out/r5g35/err.txt &&
timeout -k 10 300 python bench.py --model resnet50 --steps 20 --warmup 5 > gpurun_out/r5g35/rn50_on2.json 2>> gpurun_out/r5g35/err.txt &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5g35/prof_on -o run -- python bench.py --model resnet50 --steps 5 --warmup 3 > /dev/null 2>> gpurun_out/r5g35/err.txt &&
FF_CONV_BN_BWD=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5g35/prof_off -o run -- python bench.py --model resnet50 --steps 5 --warmup 3 > /dev/null 2>> gpurun_out/r5g35/err.txt
