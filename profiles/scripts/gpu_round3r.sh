set -o pipefail
GEMMT_DBG=0,64 timeout -k 10 400 python -u tools/gemm_ablate.py --gemmt > gpurun_out/gemm_ablate_t.jsonl 2> gpurun_out/gemm_ablate_t.err
