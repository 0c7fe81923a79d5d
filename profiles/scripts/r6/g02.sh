#!/bin/bash
# round 6, call 2: attention / LayerNorm / conv tests at the tightened bounds,
# BERT-large bench on HEAD, DLRM kernel trace with per-step boundaries at the
# loss kernel (one launch per step)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6g02; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread $R/tests/test_kernels_gpu.py -k "attention or layernorm" > $O/tests.txt 2>&1 || { tail -40 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
timeout -k 10 400 python3 $R/bench.py --steps 20 --warmup 5 > $O/bench_bert.log 2>&1 || { tail -20 $O/bench_bert.log; exit 1; }
tail -1 $O/bench_bert.log | cut -c1-300
timeout -k 10 300 python3 $R/bench.py --model dlrm --steps 50 --warmup 10 > $O/bench_dlrm.log 2>&1 || { tail -20 $O/bench_dlrm.log; exit 1; }
tail -1 $O/bench_dlrm.log | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_dlrm -o dl -- \
    python3 $R/bench.py --model dlrm --steps 20 --warmup 5 > $O/prof_dlrm.log 2>&1 || { tail -20 $O/prof_dlrm.log; exit 1; }
DB=$(find $O/prof_dlrm -name "dl_results.db" | head -n 1)
[ -n "$DB" ] && python3 $R/tools/prof_summary.py $DB --steps 10 --marker mse_kernel --top 30 > $O/dlrm_kernels.txt
head -30 $O/dlrm_kernels.txt
