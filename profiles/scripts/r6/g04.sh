#!/bin/bash
# round 6, call 4: full GPU tier + smoke on HEAD, GPT-3 medium / Inception-v3 benches
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6g04; mkdir -p $O
cd $R
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/gpu_tier.txt 2>&1
rc=$?
tail -5 $O/gpu_tier.txt
# 1 = test failures (read them afterwards); anything else (timeout, abort, fault) ends the call
[ $rc -le 1 ] || exit $rc
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 1; }
tail -2 $O/smoke.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 python3 $R/bench.py --model gpt3-medium --steps 10 --warmup 3 > $O/bench_gpt.log 2>&1 || { tail -20 $O/bench_gpt.log; exit 1; }
tail -1 $O/bench_gpt.log | cut -c1-300
timeout -k 10 400 python3 $R/bench.py --model inception-v3 --steps 10 --warmup 3 > $O/bench_inc.log 2>&1 || { tail -20 $O/bench_inc.log; exit 1; }
tail -1 $O/bench_inc.log | cut -c1-300
PYTHONPATH=$R timeout -k 10 300 python3 $R/tools/mem_audit.py resnet50 256 > $O/mem_rn50.jsonl 2>&1 || { tail -20 $O/mem_rn50.jsonl; exit 1; }
head -20 $O/mem_rn50.jsonl
PYTHONPATH=$R timeout -k 10 300 python3 $R/tools/mem_audit.py bert-large 64 > $O/mem_bert.jsonl 2>&1 || { tail -20 $O/mem_bert.jsonl; exit 1; }
head -20 $O/mem_bert.jsonl
