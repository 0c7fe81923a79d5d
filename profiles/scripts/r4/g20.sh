#!/bin/bash
# gemmt_kernel STG 2 (variant 6): reads / DMA issues interleaved with the
# MFMAs (DBG 256) vs the clustered schedule, NT input-gradient shapes (and
# NN forward: d0 there is gemmt_kk_kernel), hipBLASLt alongside
set -o pipefail
O=gpurun_out/r4g20; mkdir -p $O
for i in 1 2; do
  GEMMT_ABL_VARIANT=6 GEMMT_DBG=0,256 timeout -k 10 300 python -u tools/gemm_ablate.py --gemmt > $O/ablate_256.$i.jsonl 2>&1 || exit 1
done
cat $O/ablate_256.*.jsonl | grep '^{'
