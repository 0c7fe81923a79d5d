set -o pipefail
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "gemm or gelu or act" > gpurun_out/gemm_tests.log 2>&1 && \
timeout -k 10 400 python -u tools/gemm_ab.py --only fwd,dx --cands blaslt,t --rounds 3 > gpurun_out/gemm_ab.jsonl 2> gpurun_out/gemm_ab.err && \
FF_GEMM_REPORT=1 timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_bert.log 2> gpurun_out/bench_bert_gemm_report.txt
