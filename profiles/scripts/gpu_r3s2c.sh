# A/B: dK/dV attention kernel with all LDS fragments of a subtile prefetched (FFK_ATTN_BWD_PF=1) vs per-pair reads.
set -o pipefail
FFK_ATTN_BWD_PF=1 timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "test_attention" > gpurun_out/pf_tests.log 2>&1 || exit $?
for i in 1 2; do
  FFK_ATTN_BWD_PF=0 timeout -k 10 120 python -u tools/attn_time.py 50 >> gpurun_out/pf_ab.log 2>&1 || exit $?
  FFK_ATTN_BWD_PF=1 timeout -k 10 120 python -u tools/attn_time.py 50 >> gpurun_out/pf_ab.log 2>&1 || exit $?
done
