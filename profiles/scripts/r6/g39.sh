#!/bin/bash
# round 6, call 39: the AE protocol's searched configuration as the main run at 4 gloo ranks sharing the GPU
# (12-layer BERT-large-width, 2 sequences / rank, budget 30): the searched tensor / head splits on the HIP kernels
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6g39; mkdir -p $O
cd $R
for S in search dp; do
FF_HANG_DUMP_S=60 FF_BENCH_REHEARSAL=1 FF_DIST_BACKEND=gloo timeout -k 10 400 \
  python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29561 bench.py \
  --gpus 4 --layers 12 --batch-per-gpu 2 --budget 30 --steps 5 --warmup 2 --strategy $S --no-ae --no-dp-compare --no-calibrate \
  > $O/ae4_$S.jsonl 2> $O/ae4_$S.err
echo "4-rank AE $S rc=$?"
tail -1 $O/ae4_$S.jsonl | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); c=d['config']
print(d['value'], d['ms_per_step'], c['parallelism'][:200], c.get('graph_segments'), c.get('native_replay'), (c.get('search') or {}).get('predicted_speedup_over_dp'))"
done
