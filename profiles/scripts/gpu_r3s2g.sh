# LayerNorm backward: residual gradient loaded with the row. Tests + GPT (pre-LN, uses dres) A/B vs ab_prev.
set -o pipefail
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_fusions.py -m gpu > gpurun_out/ln_tests.log 2>&1 || exit $?
rm -f gpurun_out/ln_ab.log
for i in 1 2; do
  FF_PKG_ROOT=ab_prev timeout -k 10 300 python -u bench.py --model gpt3-medium --steps 10 --warmup 3 2>/dev/null | sed 's/^/prev /' >> gpurun_out/ln_ab.log || exit $?
  timeout -k 10 300 python -u bench.py --model gpt3-medium --steps 10 --warmup 3 2>/dev/null | sed 's/^/tree /' >> gpurun_out/ln_ab.log || exit $?
done
