#!/bin/bash
# round 6, call 49: optimizer update overlapped with the backward (FF_OVERLAP_UPDATE=1) at the round-6 batches,
# same box, interleaved (round 2 measured it neutral at 32 sequences)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6g49; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for m in bert-large gpt3-medium; do for ov in 0 1 0 1; do
  FF_OVERLAP_UPDATE=$ov timeout -k 10 300 python3 $R/bench.py --model $m --steps 10 --warmup 3 > $O/${m}_$ov.jsonl 2> $O/${m}_$ov.err || { tail -5 $O/${m}_$ov.err; exit 1; }
  tail -1 $O/${m}_$ov.jsonl | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$m', 'overlap=$ov', d['value'], d['ms_per_step'], d['config']['final_loss'])"
done; done
