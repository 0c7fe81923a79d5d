# round 4, call 13: multi-rank rehearsal of bench.py on one GPU (2 ranks share
# cuda:0 over gloo: the executor / search / bucketing / redistribution code of
# an N-GPU run) for BERT-large (reduced per-GPU batch: two ranks on one card)
# and DLRM (searched parameter-parallel tables)
set -o pipefail
mkdir -p gpurun_out/r4g13
export TMPDIR=/tmp
export FF_BENCH_REHEARSAL=1   # gloo on one GPU is allowed, the JSON line names the backend
FF_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --model bert-large --gpus 2 --steps 3 --warmup 1 \
  --batch-per-gpu 16 > gpurun_out/r4g13/bert_2rank.json 2> gpurun_out/r4g13/bert_2rank.err \
  || { tail -30 gpurun_out/r4g13/bert_2rank.err; exit 1; }
tail -1 gpurun_out/r4g13/bert_2rank.json | cut -c1-400
FF_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29518 bench.py --model dlrm --gpus 2 --steps 5 --warmup 2 \
  > gpurun_out/r4g13/dlrm_2rank.json 2> gpurun_out/r4g13/dlrm_2rank.err \
  || { tail -30 gpurun_out/r4g13/dlrm_2rank.err; exit 1; }
tail -1 gpurun_out/r4g13/dlrm_2rank.json | cut -c1-400
