#!/bin/bash
# round 4, call 18: full GPU tier with the padded-image gemmt kernel on by
# default, then end-to-end A/B of it (FFK_GEMMT_KK=1 / 0) on the BERT-large
# and GPT-3 medium bench steps, same box
set -o pipefail
O=gpurun_out/r4g18; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.txt 2>&1 \
  || { tail -30 $O/gpu_tests.txt; exit 1; }
tail -2 $O/gpu_tests.txt
for M in bert-large gpt3-medium; do
  for kk in 1 0 1 0; do
    FFK_GEMMT_KK=$kk timeout -k 10 400 python -u bench.py --model $M --steps 20 --warmup 5 > $O/bench_${M}_kk$kk.$RANDOM.log 2>&1 \
      || { tail -20 $O/bench_${M}_kk$kk.*.log; exit 1; }
  done
done
for f in $O/bench_*.log; do echo "$f $(tail -1 $f | cut -c1-150)"; done
