#!/bin/bash
# round 6, call 1: bf16 grouped convolutions on the MFMA kernels (tests at
# output-rounding bounds), tightened conv bounds, tolerance probe of attention /
# LayerNorm, ResNeXt-50 bench + kernel trace
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6g01; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
true
tail -3 $O/tests.txt
PYTHONPATH=$R timeout -k 10 200 python3 $R/tools/tol_probe.py > $O/tol_probe.jsonl 2>&1 || { tail -20 $O/tol_probe.jsonl; exit 1; }
timeout -k 10 400 python3 $R/bench.py --model resnext50 --steps 10 --warmup 3 > $O/bench_resnext50.log 2>&1 || { tail -20 $O/bench_resnext50.log; exit 1; }
tail -1 $O/bench_resnext50.log | cut -c1-400
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_rx -o rx -- \
    python3 $R/bench.py --model resnext50 --steps 3 --warmup 2 > $O/prof_rx.log 2>&1 || { tail -20 $O/prof_rx.log; exit 1; }
DB=$(find $O/prof_rx -name "rx_results.db" | head -n 1)
[ -n "$DB" ] && python3 $R/tools/prof_summary.py $DB --steps 3 --top 40 > $O/resnext50_kernels.txt
head -30 $O/resnext50_kernels.txt
