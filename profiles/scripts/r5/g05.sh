# round 5, call 5: full GPU test tier, smoke, 1-GPU BERT-large bench and a
# 2-rank gloo rehearsal of the multi-GPU path (comm calibration fields)
set -o pipefail
O=gpurun_out/r5g05; mkdir -p $O
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.txt 2>&1
rc=$?; tail -5 $O/gpu_tests.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 1; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench.jsonl 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
tail -1 $O/bench.jsonl
FF_BENCH_REHEARSAL=1 FF_DIST_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 2 --warmup 1 --batch-per-gpu 8 --no-dp-compare > $O/rehearsal.jsonl 2> $O/rehearsal.err || { tail -20 $O/rehearsal.err; exit 1; }
tail -1 $O/rehearsal.jsonl | cut -c1-1500
