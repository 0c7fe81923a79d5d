# Split-K 128-tile GEMM: numerics, then DLRM A/B vs ab_prev (no split-K candidates, framework sparse update).
set -o pipefail
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "gemm" > gpurun_out/splitk_tests.log 2>&1 || exit $?
rm -f gpurun_out/splitk_ab.log
for i in 1 2; do
  FF_PKG_ROOT=ab_prev timeout -k 10 300 python -u bench.py --model dlrm --steps 20 --warmup 5 2>/dev/null | sed 's/^/prev /' >> gpurun_out/splitk_ab.log || exit $?
  FF_GEMM_REPORT=1 timeout -k 10 300 python -u bench.py --model dlrm --steps 20 --warmup 5 2>gpurun_out/dlrm_gemm_report.txt | sed 's/^/tree /' >> gpurun_out/splitk_ab.log || exit $?
done
