# round 4, call 5: the 64x64-tile MLP GEMM (gemms.hip), the eight-wave NT GEMM
# (gemmn.hip), batched matmul and gemmt's bf16 accumulate epilogue —
# numerics first; then the input-gradient GEMM A/B on the BERT-large shapes
# (plain and accumulate), BERT-large with its autotune report, and DLRM with
# the library MLP GEMMs vs gemms (same box)
set -o pipefail
mkdir -p gpurun_out/r4g05
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
    -k "tile64 or bmm or wave128dma2 or wave128- or nt8wave" > gpurun_out/r4g05/pytest_gemms.log 2>&1 \
    || { tail -30 gpurun_out/r4g05/pytest_gemms.log; exit 1; }
tail -3 gpurun_out/r4g05/pytest_gemms.log
timeout -k 10 240 python -u tools/gemm_ab.py --only dx --cands blaslt,u,w,n --rounds 5 \
    > gpurun_out/r4g05/gemm_ab_dx.jsonl 2>&1 || exit 1
timeout -k 10 240 python -u tools/gemm_ab.py --only dx --cands blaslt,u,w,n --rounds 5 --beta 1 \
    > gpurun_out/r4g05/gemm_ab_dx_beta.jsonl 2>&1 || exit 1
FF_GEMM_REPORT=1 timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 \
    > gpurun_out/r4g05/bench_bert.json 2> gpurun_out/r4g05/bench_bert.err || exit 1
tail -1 gpurun_out/r4g05/bench_bert.json | cut -c1-200
for V in 0 1; do
  FF_GEMMS=$V timeout -k 10 240 python -u bench.py --model dlrm --steps 20 --warmup 5 \
      > gpurun_out/r4g05/bench_dlrm_gemms$V.json 2> gpurun_out/r4g05/bench_dlrm_gemms$V.err || exit 1
  tail -1 gpurun_out/r4g05/bench_dlrm_gemms$V.json | cut -c1-160
done
