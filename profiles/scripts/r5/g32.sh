#!/bin/bash
# BN finalize+apply fold: kernels test, executor test, resnet bench
set -o pipefail
mkdir -p gpurun_out/r5g32
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_gpu.py tests/test_executor_gpu.py > gpurun_out/r5g32/tests.txt 2>&1 &&
timeout -k 10 300 python bench.py --model resnet50 --steps 20 --warmup 5 > gpurun_out/r5g32/rn50.json 2> gpurun_out/r5g32/rn50.err &&
FF_BN_FUSED_FA=0 timeout -k 10 300 python bench.py --model resnet50 --steps 20 --warmup 5 > gpurun_out/r5g32/rn50_unfused.json 2>> gpurun_out/r5g32/rn50.err
