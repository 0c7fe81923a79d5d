#!/bin/bash
# round 6, call 23: what retiring rocBLAS / hipBLASLt costs today (same box): BERT-large and GPT-3 medium with and
# without library GEMM candidates, and the library-free BERT step's kernel trace
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6g23; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for i in 1 2; do
  timeout -k 10 300 python3 $R/bench.py --steps 20 --warmup 5 > $O/bert_lib_$i.log 2>&1 || { tail -20 $O/bert_lib_$i.log; exit 1; }
  FF_LIBRARY_GEMM=0 timeout -k 10 300 python3 $R/bench.py --steps 20 --warmup 5 > $O/bert_nolib_$i.log 2>&1 || { tail -20 $O/bert_nolib_$i.log; exit 1; }
done
timeout -k 10 300 python3 $R/bench.py --model gpt3-medium --steps 10 --warmup 3 > $O/gpt_lib.log 2>&1 || { tail -20 $O/gpt_lib.log; exit 1; }
FF_LIBRARY_GEMM=0 timeout -k 10 300 python3 $R/bench.py --model gpt3-medium --steps 10 --warmup 3 > $O/gpt_nolib.log 2>&1 || { tail -20 $O/gpt_nolib.log; exit 1; }
for f in bert_lib_1 bert_nolib_1 bert_lib_2 bert_nolib_2 gpt_lib gpt_nolib; do
  tail -1 $O/$f.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print('$f', d['value'], d['ms_per_step'], c['gemm_choices'])"
done
FF_LIBRARY_GEMM=0 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o nl -- \
    python3 $R/bench.py --steps 10 --warmup 3 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
DB=$(find $O/prof -name "nl_results.db" | head -n 1)
[ -n "$DB" ] && python3 $R/tools/prof_summary.py $DB --steps 5 --top 30 > $O/bert_nolib_kernels.txt
head -25 $O/bert_nolib_kernels.txt
