# round 5, call 11: the C API GPU backing with conv / batch norm / pooling
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5g11; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_runtime_c_gpu.py > $O/tests.txt 2>&1
rc=$?; tail -5 $O/tests.txt
timeout -k 10 120 ./bin/ffc-runtime-c-test > $O/capi_gpu.txt 2>&1; grep -i "device\|PASSED\|FAIL" $O/capi_gpu.txt
FF_C_API_DEVICE=cpu timeout -k 10 120 ./bin/ffc-runtime-c-test > $O/capi_cpu.txt 2>&1; grep -i "parity" $O/capi_cpu.txt
exit $rc
