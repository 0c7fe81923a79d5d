#!/bin/bash
# BN backward sums from the consuming conv's dgrad epilogue: tests + ResNet A/B
set -o pipefail
mkdir -p gpurun_out/r5g34
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_gpu.py tests/test_executor_gpu.py > gpurun_out/r5g34/tests.txt 2>&1 &&
timeout -k 10 300 python bench.py --model resnet50 --steps 20 --warmup 5 > gpurun_out/r5g34/rn50.json 2> gpurun_out/r5g34/rn50.err &&
FF_CONV_BN_BWD=0 timeout -k 10 300 python bench.py --model resnet50 --steps 20 --warmup 5 > gpurun_out/r5g34/rn50_off.json 2>> gpurun_out/r5g34/rn50.err &&
timeout -k 10 300 python bench.py --model resnet50 --steps 20 --warmup 5 > gpurun_out/r5g34/rn50_2.json 2>> gpurun_out/r5g34/rn50.err
