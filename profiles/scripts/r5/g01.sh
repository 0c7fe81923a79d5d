#!/bin/bash
# round 5, call 1: exact-fp32 MFMA kernels (igemm32.hip) numerics + fp32 model
set -o pipefail
mkdir -p gpurun_out/r5
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_igemm32_gpu.py tests/test_fp32_model_gpu.py > gpurun_out/r5/g01_tests.txt 2>&1
rc=$?
tail -5 gpurun_out/r5/g01_tests.txt
exit $rc
