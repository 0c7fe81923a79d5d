#!/bin/bash
# round 6, call 35: 2 and 4 gloo ranks sharing the GPU through the whole bench flow on HEAD (search keeps DP below a
# 2 % predicted gain; AE protocol in child jobs with a progress line every 30 s)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6g35; mkdir -p $O
cd $R
show() { tail -1 $1 | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); c=d['config']
print(d['value'], d['ms_per_step'], d['world_size'], d['backend'], c['parallelism'][:60], c.get('graph_segments'), c.get('native_replay'))
for k in ('speedup_over_dp','dp_reference','ae_bert','ae_speedup_over_dp','after_headline'):
    print(' ', k, json.dumps(c.get(k))[:500])"; }
for N in 2 4; do
  FF_BENCH_REHEARSAL=1 FF_DIST_BACKEND=gloo FF_MEM_PHASES=1 timeout -k 10 560 python3 -m torch.distributed.run --nnodes=1 \
    --nproc-per-node $N --master-addr 127.0.0.1 --master-port 2953$N bench.py --gpus $N --steps 3 --warmup 1 --batch-per-gpu 16 \
    > $O/gloo$N.jsonl 2> $O/gloo$N.err
  echo "gloo $N-rank rc=$?"; show $O/gloo$N.jsonl
done
