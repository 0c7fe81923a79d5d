#!/bin/bash
# round 6, call 26 (27: per-step times): 2-rank rehearsal (gloo, one GPU): memory through search run -> release -> DP reference,
# after emptying the eager cache before the segmented capture
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6g27; mkdir -p $O
cd $R
FF_BENCH_REHEARSAL=1 FF_DIST_BACKEND=gloo FF_MEM_PHASES=1 FF_STEP_TIMES=1 timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29522 bench.py --gpus 2 --steps 3 --warmup 1 --no-ae --no-calibrate \
  > $O/r2.jsonl 2> $O/r2.err || { tail -30 $O/r2.err; exit 1; }
grep "\[mem\]\|\[step\]" $O/r2.err | cut -c1-200
tail -1 $O/r2.jsonl | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print(d['value'], d['ms_per_step'], c['parallelism'], c.get('graph_segments'), c.get('dp_samples_per_sec'), c.get('speedup_over_dp'))"
