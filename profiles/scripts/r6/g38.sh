#!/bin/bash
# round 6, call 38: 4 gloo ranks sharing the GPU -- headline (batch 16 / rank) + the AE protocol's child jobs at
# 4 ranks (2 sequences / rank: the searched tensor / head splits), stacks every 60 s
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6g38; mkdir -p $O
cd $R
FF_HANG_DUMP_S=60 FF_BENCH_CHILD_LOG_DIR=$O/children FF_BENCH_REHEARSAL=1 FF_DIST_BACKEND=gloo timeout -k 10 800 \
  python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29551 bench.py \
  --gpus 4 --steps 3 --warmup 1 --batch-per-gpu 16 --no-dp-compare --no-calibrate > $O/gloo4.jsonl 2> $O/gloo4.err
echo "gloo 4-rank rc=$?"
tail -1 $O/gloo4.jsonl | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); c=d['config']
print(d['value'], d['ms_per_step'], c['parallelism'][:80])
for k in ('speedup_over_dp','dp_reference','ae_bert','ae_speedup_over_dp','after_headline'):
    print(' ', k, json.dumps(c.get(k))[:600])"
