#!/bin/bash
# round 6, call 48: library-free GEMMs at the round-6 defaults (BERT-large 128, GPT-3 medium 32), same box, interleaved
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6g48; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for m in bert-large gpt3-medium; do for lib in 1 0 1 0; do
  FF_LIBRARY_GEMM=$lib timeout -k 10 300 python3 $R/bench.py --model $m --steps 10 --warmup 3 > $O/${m}_$lib.jsonl 2> $O/${m}_$lib.err || { tail -5 $O/${m}_$lib.err; exit 1; }
  tail -1 $O/${m}_$lib.jsonl | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$m', 'library' if $lib else 'library-free', d['value'], d['ms_per_step'])"
done; done
