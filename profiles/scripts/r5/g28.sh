# round 5, call 28: final GPU tier + four benches + BERT / ResNet-50 kernel traces at HEAD
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5g28; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests > $O/tests.txt 2>&1
rc=$?; tail -3 $O/tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --model resnet50 --steps 20 --warmup 5 > $O/bench_rn.jsonl 2>&1 || { tail -20 $O/bench_rn.jsonl; exit 1; }
tail -1 $O/bench_rn.jsonl | cut -c1-200
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_bert.jsonl 2>&1 || { tail -20 $O/bench_bert.jsonl; exit 1; }
tail -1 $O/bench_bert.jsonl | cut -c1-200
timeout -k 10 300 python bench.py --model gpt3-medium --steps 10 --warmup 3 > $O/bench_gpt.jsonl 2>&1 || { tail -20 $O/bench_gpt.jsonl; exit 1; }
tail -1 $O/bench_gpt.jsonl | cut -c1-200
timeout -k 10 300 python bench.py --model dlrm --steps 50 --warmup 10 > $O/bench_dlrm.jsonl 2>&1 || { tail -20 $O/bench_dlrm.jsonl; exit 1; }
tail -1 $O/bench_dlrm.jsonl | cut -c1-200
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt | cut -c1-200
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_rn -o rn -- \
    python3 $R/bench.py --model resnet50 --steps 5 --warmup 3 > $O/prof_rn.log 2>&1 || { tail -20 $O/prof_rn.log; exit 1; }
DB=$(find $O/prof_rn -name "rn_results.db" | head -n 1)
[ -n "$DB" ] && python3 $R/tools/prof_summary.py $DB --steps 5 --top 40 > $O/rn50_kernels.txt
head -12 $O/rn50_kernels.txt
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_bert -o bert -- \
    python3 $R/bench.py --steps 5 --warmup 3 > $O/prof_bert.log 2>&1 || { tail -20 $O/prof_bert.log; exit 1; }
DB=$(find $O/prof_bert -name "bert_results.db" | head -n 1)
[ -n "$DB" ] && python3 $R/tools/prof_summary.py $DB --steps 5 --top 40 > $O/bert_kernels.txt
head -12 $O/bert_kernels.txt
