#!/bin/bash
# padded-image gemmt_kk_kernel (A^T B and A B): numerics, then A/B vs the
# swizzled-image gemmt_kernel (FFK_GEMMT_KK=0) on the BERT-large shapes
set -o pipefail
O=gpurun_out/r4g17; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  -k "test_gemmp and (False-False or True-False) and wave128dma2" > $O/pytest_kk.txt 2>&1 || { tail -30 $O/pytest_kk.txt; exit 1; }
tail -3 $O/pytest_kk.txt
for kk in 1 0 1 0; do  # 1 = padded kernel
  FFK_GEMMT_KK=$kk timeout -k 10 240 python -u tools/gemm_ab.py --only fwd,dw --cands w --rounds 5 --iters 10 \
    > $O/ab_kk$kk.$RANDOM.jsonl 2>&1 || exit 1
done
ls $O
