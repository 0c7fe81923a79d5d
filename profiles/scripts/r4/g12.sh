# round 4, call 12: how much of gemmt's LDS-DMA forms is exposed load latency
# (DBG 128 skips the wait for the next K-tile's DMA; results garbage, time only)
set -o pipefail
mkdir -p gpurun_out/r4g12
for V in 6 4; do
  GEMMT_ABL_VARIANT=$V GEMMT_DBG=0,128,8,136 timeout -k 10 300 python -u tools/gemm_ablate.py --gemmt \
      > gpurun_out/r4g12/ablate_v$V.jsonl 2> gpurun_out/r4g12/ablate_v$V.err || { tail -5 gpurun_out/r4g12/ablate_v$V.err; exit 1; }
  cat gpurun_out/r4g12/ablate_v$V.jsonl
done
