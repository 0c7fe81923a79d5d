#!/bin/bash
# round 6, call 37: BERT-large and GPT-3 medium kernel traces on HEAD (per-step summaries of the last 5 steps)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6g37; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for m in bert-large gpt3-medium; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_$m -o k -- \
      python3 $R/bench.py --model $m --steps 10 --warmup 3 > $O/prof_$m.log 2>&1 || { tail -20 $O/prof_$m.log; exit 1; }
  DB=$(find $O/prof_$m -name "k_results.db" | head -n 1)
  [ -n "$DB" ] && python3 $R/tools/prof_summary.py $DB --steps 5 --top 40 > $O/${m}_kernels.txt
  head -22 $O/${m}_kernels.txt
  rm -rf $O/prof_$m
done
