# A/B: q/k/v bias gradients inside the attention backward (slab partials) vs the separate colsum pass, batch-64 BERT-large.
set -o pipefail
FF_ATTN_FUSED_DBIAS=1 timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "attention" > gpurun_out/dbias_tests.log 2>&1 || exit $?
bash tools/ab_env.sh FF_ATTN_FUSED_DBIAS "--steps 10 --warmup 3" ab_dbias_b64
