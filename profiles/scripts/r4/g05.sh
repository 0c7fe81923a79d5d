# round 4, call 5: the 64x64-tile MLP GEMM (gemms.hip), batched matmul and
# gemmt's bf16 accumulate epilogue — numerics first; then same-box benches
# (BERT-large with its GEMM autotune report, DLRM library MLP GEMMs vs gemms);
# then the simulator-calibration inputs (g04.sh)
set -o pipefail
mkdir -p gpurun_out/r4g05
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
    -k "tile64 or bmm or wave128dma2 or wave128-" > gpurun_out/r4g05/pytest_gemms.log 2>&1 \
    || { tail -30 gpurun_out/r4g05/pytest_gemms.log; exit 1; }
tail -3 gpurun_out/r4g05/pytest_gemms.log
FF_GEMM_REPORT=1 timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 \
    > gpurun_out/r4g05/bench_bert.json 2> gpurun_out/r4g05/bench_bert.err || exit 1
tail -1 gpurun_out/r4g05/bench_bert.json | cut -c1-200
for V in 0 1; do
  FF_GEMMS=$V timeout -k 10 240 python -u bench.py --model dlrm --steps 20 --warmup 5 \
      > gpurun_out/r4g05/bench_dlrm_gemms$V.json 2> gpurun_out/r4g05/bench_dlrm_gemms$V.err || exit 1
  tail -1 gpurun_out/r4g05/bench_dlrm_gemms$V.json | cut -c1-160
done
MODELS="bert-large dlrm gpt3-medium resnet50" bash profiles/scripts/r4/g04.sh
