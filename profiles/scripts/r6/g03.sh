#!/bin/bash
# round 6, call 3: the C API GPU backing with the BERT parity program
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6g03; mkdir -p $O
cd $R
timeout -k 10 200 ./bin/ffc-runtime-c-test > $O/capi_gpu.txt 2>&1 || { tail -30 $O/capi_gpu.txt; exit 1; }
grep parity $O/capi_gpu.txt
FF_C_API_DEVICE=cpu timeout -k 10 200 ./bin/ffc-runtime-c-test > $O/capi_cpu.txt 2>&1 || { tail -30 $O/capi_cpu.txt; exit 1; }
grep parity $O/capi_cpu.txt
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_runtime_c_gpu.py > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
