set -o pipefail
FF_GEMM_REPORT=1 timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_bert.log 2> gpurun_out/bench_bert_gemm_report.txt && \
timeout -k 10 400 python -u bench.py --model gpt3-medium --steps 10 --warmup 3 > gpurun_out/bench_gpt.log 2>&1
