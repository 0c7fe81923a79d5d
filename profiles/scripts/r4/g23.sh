#!/bin/bash
# gemmt_kk_kernel for A B^T (FFK_GEMMT_KK_NT=1): numerics of the NT cases,
# GEMM A/B on the BERT-large input-gradient shapes next to hipBLASLt, bench A/B
set -o pipefail
O=gpurun_out/r4g23; mkdir -p $O
FFK_GEMMT_KK_NT=1 timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  -k "test_gemmp and False-True and wave128dma2" > $O/pytest_nt.txt 2>&1 || { tail -30 $O/pytest_nt.txt; exit 1; }
tail -2 $O/pytest_nt.txt
for nt in 1 0 1 0; do
  FFK_GEMMT_KK_NT=$nt timeout -k 10 240 python -u tools/gemm_ab.py --only dx --cands w,blaslt --rounds 5 --iters 10 \
    > $O/ab_nt$nt.$RANDOM.jsonl 2>&1 || exit 1
  FFK_GEMMT_KK_NT=$nt timeout -k 10 240 python -u tools/gemm_ab.py --only dx --cands w,blaslt --rounds 5 --iters 10 --beta 1 \
    > $O/ab_nt_beta$nt.$RANDOM.jsonl 2>&1 || exit 1
done
for nt in 1 0 1 0; do
  FFK_GEMMT_KK_NT=$nt timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $O/bench_bert_nt$nt.$RANDOM.log 2>&1 || exit 1
done
for f in $O/bench_*.log; do echo "$f $(tail -1 $f | cut -c1-120)"; done
