set -o pipefail
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "test_gemmp or test_attention" > gpurun_out/gemm_tests.log 2>&1 && \
FF_GEMM_REPORT=1 timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_bert.log 2> gpurun_out/bench_bert_gemm_report.txt && \
FF_ATTN_FUSED_DBIAS=0 timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_bert_nofuse.log 2>&1 && \
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_bert2.log 2>&1
