# Graph-timed autotuning of small GEMM / conv candidates: GEMM + conv tests, then DLRM / ResNet-50 / BERT benches.
set -o pipefail
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_sparse_update.py -m gpu > gpurun_out/gt_tests.log 2>&1 || exit $?
FF_GEMM_REPORT=1 timeout -k 10 300 python -u bench.py --model dlrm --steps 20 --warmup 5 > gpurun_out/gt_dlrm.log 2> gpurun_out/gt_dlrm_report.txt || exit $?
timeout -k 10 300 python -u bench.py --model dlrm --steps 20 --warmup 5 >> gpurun_out/gt_dlrm.log 2>/dev/null || exit $?
timeout -k 10 400 python -u bench.py --model resnet50 --steps 20 --warmup 5 > gpurun_out/gt_resnet.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > gpurun_out/gt_bert.log 2>&1
