#!/bin/bash
# round 5, call 41: default FFK_BN_RED_BLOCKS=1024 -- conv/BN GPU tests + ResNet-50 bench
set -o pipefail
O=gpurun_out/r5g41; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_gpu.py tests/test_executor_gpu.py > $O/tests.txt 2>&1 &&
timeout -k 10 300 python bench.py --model resnet50 --steps 20 --warmup 5 > $O/rn50.json 2> $O/err.txt
