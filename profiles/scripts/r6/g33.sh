#!/bin/bash
# round 6, call 33: multi-rank bench flow with the DP reference and the AE protocol in isolated child jobs (other ranks wait on the store), explicit process-group
# shutdown -- over RCCL at world 1, then 2 gloo ranks sharing the GPU (BERT-large, default batch)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6g33; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
show() { tail -1 $1 | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); c=d['config']
print(d['value'], d['ms_per_step'], d['world_size'], d['backend'], c['parallelism'][:60], c.get('graph_segments'), c.get('native_replay'))
for k in ('speedup_over_dp','dp_samples_per_sec','dp_reference','ae_bert','ae_speedup_over_dp','after_headline'):
    print(' ', k, json.dumps(c.get(k))[:500])"; }
FF_DIST_WORLD1=1 FF_BENCH_REHEARSE_MULTI=1 timeout -k 10 500 python3 $R/bench.py --steps 10 --warmup 3 > $O/rccl1.jsonl 2> $O/rccl1.err
echo "rccl world-1 rc=$?"; show $O/rccl1.jsonl
cd $R
FF_BENCH_REHEARSAL=1 FF_DIST_BACKEND=gloo timeout -k 10 500 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29524 bench.py --gpus 2 --steps 3 --warmup 1 > $O/gloo2.jsonl 2> $O/gloo2.err
echo "gloo 2-rank rc=$?"; show $O/gloo2.jsonl
