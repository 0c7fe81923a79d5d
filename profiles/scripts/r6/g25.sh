#!/bin/bash
# round 6, call 25: why the 2-rank (gloo, one GPU) DP reference ran 12x slower than the near-DP searched strategy
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6g25; mkdir -p $O
cd $R
for S in dp search; do
  FF_BENCH_REHEARSAL=1 FF_DIST_BACKEND=gloo FF_MEM_PHASES=1 timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29521 bench.py --gpus 2 --steps 3 --warmup 1 --strategy $S --no-ae --no-calibrate --no-dp-compare \
    > $O/r2_$S.jsonl 2> $O/r2_$S.err || { tail -30 $O/r2_$S.err; exit 1; }
  grep "\[mem\]" $O/r2_$S.err | cut -c1-200 | head -8
  tail -1 $O/r2_$S.jsonl | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print('$S', d['value'], d['ms_per_step'], c['parallelism'], c.get('hipgraph'), c.get('graph_segments'), c.get('native_replay'))"
done
