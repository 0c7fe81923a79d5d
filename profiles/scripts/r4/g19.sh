#!/bin/bash
# gemmt_kk_kernel: interleaved group schedule (FFK_GEMMT_KK_SCHED=1) vs the
# clustered one (0): numerics of the interleaved form, then GEMM A/B on the
# BERT-large shapes and the bench step
set -o pipefail
O=gpurun_out/r4g19; mkdir -p $O
FFK_GEMMT_KK_SCHED=1 timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  -k "test_gemmp and (False-False or True-False) and wave128dma2" > $O/pytest_sched1.txt 2>&1 || { tail -30 $O/pytest_sched1.txt; exit 1; }
tail -2 $O/pytest_sched1.txt
for sc in 1 0 1 0; do
  FFK_GEMMT_KK_SCHED=$sc timeout -k 10 240 python -u tools/gemm_ab.py --only fwd,dw --cands w --rounds 5 --iters 10 \
    > $O/ab_sched$sc.$RANDOM.jsonl 2>&1 || exit 1
done
for sc in 1 0 1 0; do
  FFK_GEMMT_KK_SCHED=$sc timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $O/bench_bert_sched$sc.$RANDOM.log 2>&1 || exit 1
done
for f in $O/bench_*.log; do echo "$f $(tail -1 $f | cut -c1-120)"; done
