set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "test_gemmp" -x -q --timeout 60 --timeout-method thread > gpurun_out/gemmp_tests.log 2>&1 && \
timeout -k 10 600 python -u tools/gemm_ab.py --rounds 3 --iters 10 --cands blaslt,t,u > gpurun_out/gemm_ab.jsonl 2> gpurun_out/gemm_ab.err && \
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_bert.log 2>&1 && \
timeout -k 10 400 python -u bench.py --model gpt3-medium --steps 10 --warmup 3 > gpurun_out/bench_gpt.log 2>&1
