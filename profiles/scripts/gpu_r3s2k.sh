# Native row-sparse SGD: tests, then DLRM A/B against the previous package snapshot (framework path).
set -o pipefail
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_sparse_update.py tests/test_kernels_gpu.py -m gpu > gpurun_out/sparse_tests.log 2>&1 || exit $?
rm -f gpurun_out/sparse_ab.log
for i in 1 2; do
  FF_PKG_ROOT=ab_prev timeout -k 10 300 python -u bench.py --model dlrm --steps 20 --warmup 5 2>/dev/null | sed 's/^/prev /' >> gpurun_out/sparse_ab.log || exit $?
  timeout -k 10 300 python -u bench.py --model dlrm --steps 20 --warmup 5 2>/dev/null | sed 's/^/tree /' >> gpurun_out/sparse_ab.log || exit $?
done
