# round 5, call 12 (re-entry): rebuilt tree -> full GPU tier, BERT + ResNet-50 bench
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5g12; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests > $O/tests.txt 2>&1
rc=$?; tail -3 $O/tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_bert.jsonl 2>&1 || { tail -20 $O/bench_bert.jsonl; exit 1; }
tail -1 $O/bench_bert.jsonl | cut -c1-400
timeout -k 10 300 python bench.py --model resnet50 --steps 20 --warmup 5 > $O/bench_rn.jsonl 2>&1 || { tail -20 $O/bench_rn.jsonl; exit 1; }
tail -1 $O/bench_rn.jsonl | cut -c1-300
