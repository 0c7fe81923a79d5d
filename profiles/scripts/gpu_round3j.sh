set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -k "test_gemmp and wave128" -x -q --timeout 60 --timeout-method thread > gpurun_out/gemmp_tests.log 2>&1 && \
timeout -k 10 400 python -u tools/gemm_ablate.py --gemmt > gpurun_out/gemm_ablate_t.jsonl 2> gpurun_out/gemm_ablate_t.err
