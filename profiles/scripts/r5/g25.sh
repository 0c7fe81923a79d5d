# round 5, call 25: full GPU tier + the four bench configs at HEAD (after the conv / gemmpp work)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5g25; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests > $O/tests.txt 2>&1
rc=$?; tail -3 $O/tests.txt; [ $rc -eq 0 ] || exit $rc
FF_AUTOTUNE_REPORT=$O/autotune_bert.txt timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_bert.jsonl 2>&1 || { tail -20 $O/bench_bert.jsonl; exit 1; }
tail -1 $O/bench_bert.jsonl | cut -c1-700
timeout -k 10 300 python bench.py --model resnet50 --steps 20 --warmup 5 > $O/bench_rn.jsonl 2>&1 || { tail -20 $O/bench_rn.jsonl; exit 1; }
tail -1 $O/bench_rn.jsonl | cut -c1-200
timeout -k 10 300 python bench.py --model gpt3-medium --steps 10 --warmup 3 > $O/bench_gpt.jsonl 2>&1 || { tail -20 $O/bench_gpt.jsonl; exit 1; }
tail -1 $O/bench_gpt.jsonl | cut -c1-200
timeout -k 10 300 python bench.py --model dlrm --steps 50 --warmup 10 > $O/bench_dlrm.jsonl 2>&1 || { tail -20 $O/bench_dlrm.jsonl; exit 1; }
tail -1 $O/bench_dlrm.jsonl | cut -c1-200
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 1; }
tail -2 $O/smoke.txt
