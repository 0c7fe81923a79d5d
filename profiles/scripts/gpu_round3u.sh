set -o pipefail
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "test_gemmp" > gpurun_out/gemm_tests.log 2>&1 && \
timeout -k 10 600 python -u tools/gemm_ab.py --rounds 3 --cands blaslt,t,u,w --only fwd,dx > gpurun_out/gemm_ab.jsonl 2> gpurun_out/gemm_ab.err
