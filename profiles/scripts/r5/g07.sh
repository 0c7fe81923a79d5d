# round 5, call 7: GPU tier (incl. the C API GPU backing), smoke, BERT-large
# bench with the native-preferring autotuner + memory record, DLRM and
# ResNet-50 benches, BERT kernel trace
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5g07; mkdir -p $O
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.txt 2>&1
rc=$?; tail -4 $O/gpu_tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/attn_time.py --xcd-ab > $O/attn_xcd_ab.jsonl 2>&1 || { tail -20 $O/attn_xcd_ab.jsonl; exit 1; }
cat $O/attn_xcd_ab.jsonl | grep shape
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 1; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_bert.jsonl 2> $O/bench_bert.err || { tail -20 $O/bench_bert.err; exit 1; }
tail -1 $O/bench_bert.jsonl | cut -c1-900
timeout -k 10 300 python bench.py --model dlrm --steps 50 --warmup 10 > $O/bench_dlrm.jsonl 2>&1 || { tail -20 $O/bench_dlrm.jsonl; exit 1; }
tail -1 $O/bench_dlrm.jsonl | cut -c1-300
timeout -k 10 300 python bench.py --model resnet50 --steps 20 --warmup 5 > $O/bench_rn50.jsonl 2>&1 || { tail -20 $O/bench_rn50.jsonl; exit 1; }
tail -1 $O/bench_rn50.jsonl | cut -c1-300
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_bert -o bert -- \
    python3 $R/bench.py --steps 5 --warmup 3 > $O/prof_bert.log 2>&1 || { tail -20 $O/prof_bert.log; exit 1; }
DB=$(find $O/prof_bert -name "bert_results.db" | head -n 1)
[ -n "$DB" ] && python3 $R/tools/prof_summary.py $DB --steps 5 --top 30 > $O/bert_kernels.txt
head -34 $O/bert_kernels.txt
