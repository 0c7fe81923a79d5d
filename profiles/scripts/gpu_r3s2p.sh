# Graph-timed autotuning without the allocator flush: tests, BERT A/B, DLRM.
set -o pipefail
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k gemm -m gpu > gpurun_out/gt2_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --model dlrm --steps 20 --warmup 5 > gpurun_out/gt2_dlrm.log 2>/dev/null || exit $?
bash tools/ab_env.sh FF_AUTOTUNE_GRAPH "--steps 10 --warmup 3" ab_autotune_graph2_bert
