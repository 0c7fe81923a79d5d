# round 5, call 9: the RCCL code path at world 1 (FF_DIST_WORLD1: nccl process
# group, graph segments cut at every collective), GPT-3 medium bench + trace
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5g09; mkdir -p $O
FF_DIST_WORLD1=1 timeout -k 10 400 python bench.py --steps 5 --warmup 3 > $O/bench_bert_nccl_w1.jsonl 2> $O/bench_bert_nccl_w1.err || { tail -30 $O/bench_bert_nccl_w1.err; exit 1; }
tail -1 $O/bench_bert_nccl_w1.jsonl | cut -c1-600
timeout -k 10 400 python bench.py --model gpt3-medium --steps 10 --warmup 3 > $O/bench_gpt.jsonl 2> $O/bench_gpt.err || { tail -20 $O/bench_gpt.err; exit 1; }
tail -1 $O/bench_gpt.jsonl | cut -c1-600
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_gpt -o gpt -- \
    python3 $R/bench.py --model gpt3-medium --steps 5 --warmup 3 > $O/prof_gpt.log 2>&1 || { tail -20 $O/prof_gpt.log; exit 1; }
DB=$(find $O/prof_gpt -name "gpt_results.db" | head -n 1)
[ -n "$DB" ] && python3 $R/tools/prof_summary.py $DB --steps 5 --top 30 > $O/gpt_kernels.txt
head -34 $O/gpt_kernels.txt
