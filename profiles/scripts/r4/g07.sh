# round 4, call 7: the software-pipelined attention forward and the delta pass
# fused into the dQ kernel (numerics, then same-process A/Bs at the BERT-large / GPT-3-medium bench shapes), then the
# in-situ per-operator costs for the simulator calibration (g06.sh)
set -o pipefail
mkdir -p gpurun_out/r4g07
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
    -k "pipelined or attention_fwd_bwd or fused_delta" > gpurun_out/r4g07/pytest_attn.log 2>&1 \
    || { tail -30 gpurun_out/r4g07/pytest_attn.log; exit 1; }
tail -2 gpurun_out/r4g07/pytest_attn.log
timeout -k 10 200 python -u tools/attn_time.py --pipe-ab > gpurun_out/r4g07/attn_pipe_ab.jsonl 2>&1 || exit 1
cat gpurun_out/r4g07/attn_pipe_ab.jsonl
timeout -k 10 200 python -u tools/attn_time.py --delta-ab > gpurun_out/r4g07/attn_delta_ab.jsonl 2>&1 || exit 1
cat gpurun_out/r4g07/attn_delta_ab.jsonl
bash profiles/scripts/r4/g06.sh
# same-box step times of the four configs (the in-situ tables' reference)
for M in bert-large gpt3-medium resnet50 dlrm; do
  timeout -k 10 300 python -u bench.py --model $M --strategy dp --no-dp-compare --steps 10 --warmup 3 \
      > gpurun_out/calib/bench_$M.json 2> gpurun_out/calib/bench_$M.err || exit 1
  tail -1 gpurun_out/calib/bench_$M.json | cut -c1-160
done
