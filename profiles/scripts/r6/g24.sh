#!/bin/bash
# round 6, call 24: the N > 1 bench flow rehearsed on one GPU (gloo ranks sharing cuda:0): BERT-large, 2 and 4 ranks,
# default per-GPU batch, search + headline + calibration + DP reference + AE protocol
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6g24; mkdir -p $O
cd $R
for N in 2 4; do
  FF_BENCH_REHEARSAL=1 FF_DIST_BACKEND=gloo timeout -k 10 540 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $N \
    --master-addr 127.0.0.1 --master-port 2951$N bench.py --gpus $N --steps 3 --warmup 1 > $O/rehearse_$N.jsonl 2> $O/rehearse_$N.err \
    || { tail -30 $O/rehearse_$N.err; exit 1; }
  tail -1 $O/rehearse_$N.jsonl | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print($N, d['value'], d['ms_per_step'], c['parallelism'], c.get('graph_segments'), c.get('native_replay'), c.get('speedup_over_dp'), c.get('ae_speedup_over_dp'), json.dumps(c.get('search'))[:300], str(c.get('ae_bert'))[:300])"
done
