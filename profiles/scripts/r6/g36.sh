#!/bin/bash
# round 6, call 36: diagnose (a) the child jobs aborting after a 2-rank batch-16 hybrid headline (their stderr kept),
# (b) 4 gloo ranks stalling after the first eager step (every rank's stacks every 60 s)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6g36; mkdir -p $O
cd $R
FF_BENCH_CHILD_LOG_DIR=$O/children FF_BENCH_REHEARSAL=1 FF_DIST_BACKEND=gloo timeout -k 10 400 python3 -m torch.distributed.run \
  --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 2 --steps 3 --warmup 1 \
  --batch-per-gpu 16 > $O/gloo2.jsonl 2> $O/gloo2.err
echo "gloo 2-rank rc=$?"
for f in $O/children/*.err; do echo "== $f"; grep -v "socket.cpp\|amdgpu.ids" $f | grep -i -B2 -A8 "error\|terminate\|abort\|Traceback" | head -40; done
FF_HANG_DUMP_S=60 FF_MEM_PHASES=1 FF_BENCH_REHEARSAL=1 FF_DIST_BACKEND=gloo timeout -k 10 400 python3 -m torch.distributed.run \
  --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29542 bench.py --gpus 4 --steps 3 --warmup 1 \
  --batch-per-gpu 16 --no-ae --no-dp-compare --no-calibrate > $O/gloo4.jsonl 2> $O/gloo4.err
echo "gloo 4-rank rc=$?"
tail -1 $O/gloo4.jsonl | cut -c1-200
