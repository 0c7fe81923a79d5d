# A/B of the attention backward fixes: ab_prev = previous build; tree PF=0 / PF=1.
set -o pipefail
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "test_attention" > gpurun_out/attn_tests.log 2>&1 || exit $?
FFK_ATTN_BWD_PF=1 timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "test_attention" >> gpurun_out/attn_tests.log 2>&1 || exit $?
rm -f gpurun_out/attn_ab.log
for i in 1 2; do
  FF_PKG_ROOT=ab_prev FFK_ATTN_BWD_PF=0 timeout -k 10 120 python -u tools/attn_time.py 50 2>/dev/null | sed 's/^/prev  /' >> gpurun_out/attn_ab.log || exit $?
  FFK_ATTN_BWD_PF=0 timeout -k 10 120 python -u tools/attn_time.py 50 2>/dev/null | sed 's/^/pf0   /' >> gpurun_out/attn_ab.log || exit $?
  FFK_ATTN_BWD_PF=1 timeout -k 10 120 python -u tools/attn_time.py 50 2>/dev/null | sed 's/^/pf1   /' >> gpurun_out/attn_ab.log || exit $?
done
