# round 4, call 7: the software-pipelined attention forward (numerics, then a
# same-process A/B at the BERT-large / GPT-3-medium bench shapes), then the
# in-situ per-operator costs for the simulator calibration (g06.sh)
set -o pipefail
mkdir -p gpurun_out/r4g07
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
    -k "pipelined or attention_fwd_bwd" > gpurun_out/r4g07/pytest_attn.log 2>&1 \
    || { tail -30 gpurun_out/r4g07/pytest_attn.log; exit 1; }
tail -2 gpurun_out/r4g07/pytest_attn.log
timeout -k 10 200 python -u tools/attn_time.py --pipe-ab > gpurun_out/r4g07/attn_pipe_ab.jsonl 2>&1 || exit 1
cat gpurun_out/r4g07/attn_pipe_ab.jsonl
bash profiles/scripts/r4/g06.sh
