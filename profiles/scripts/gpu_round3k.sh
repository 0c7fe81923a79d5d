set -o pipefail
timeout -k 10 400 python -u tools/gemm_ablate.py --gemmt > gpurun_out/gemm_ablate_t.jsonl 2> gpurun_out/gemm_ablate_t.err && \
FF_GEMM_REPORT=1 timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_bert.log 2> gpurun_out/bench_bert_gemm_report.txt
