#!/bin/bash
# gemmt_kk_kernel: reads one group ahead (FFK_GEMMT_KK_SCHED=3) vs SCH 1:
# numerics, GEMM
# A/B on the BERT-large shapes, bench A/B
set -o pipefail
O=gpurun_out/r4g28; mkdir -p $O
FFK_GEMMT_KK_SCHED=3 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  -k "test_gemmp and wave128dma2" > $O/pytest_sched3.txt 2>&1 || { tail -30 $O/pytest_sched3.txt; exit 1; }
tail -1 $O/pytest_sched3.txt
for sc in 3 1 3 1; do
  FFK_GEMMT_KK_SCHED=$sc timeout -k 10 300 python -u tools/gemm_ab.py --only fwd,dx,dw --cands w --rounds 5 --iters 10 \
    > $O/ab_sched$sc.$RANDOM.jsonl 2>&1 || exit 1
done
for sc in 3 1 3 1; do
  FFK_GEMMT_KK_SCHED=$sc timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $O/bench_bert_sched$sc.$RANDOM.log 2>&1 || exit 1
done
for f in $O/bench_*.log; do echo "$f $(tail -1 $f | cut -c1-120)"; done
