#!/bin/bash
# tightened GEMM / embedding tolerances: kernels GPU tests
set -o pipefail
mkdir -p gpurun_out/r5g33
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py > gpurun_out/r5g33/tests.txt 2>&1
