# After multi-piece concat/split and eager conv tuning: tensorops tests, ResNet-50 (bounded), DLRM, BERT.
set -o pipefail
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_tensorops_gpu.py tests/test_kernels_gpu.py -m gpu > gpurun_out/r_tests.log 2>&1 || exit $?
timeout -k 10 170 python -u bench.py --model resnet50 --steps 20 --warmup 5 > gpurun_out/r_resnet.log 2>&1 || exit $?
timeout -k 10 170 python -u bench.py --model dlrm --steps 20 --warmup 5 > gpurun_out/r_dlrm.log 2>&1 || exit $?
timeout -k 10 170 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r_bert.log 2>&1 || exit $?
timeout -k 10 170 python -u bench.py --model gpt3-medium --steps 10 --warmup 3 > gpurun_out/r_gpt.log 2>&1
