# round 4, call 24: GPU tier + smoke + the four bench configs at HEAD
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4g24; mkdir -p $O
cd $R && timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.txt 2>&1 \
  || { tail -30 $O/gpu_tests.txt; exit 1; }
tail -1 $O/gpu_tests.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
for M in bert-large gpt3-medium resnet50 dlrm; do
  timeout -k 10 400 python3 bench.py --model $M --steps 20 --warmup 5 > $O/bench_$M.log 2>&1 || { tail -20 $O/bench_$M.log; exit 1; }
  tail -1 $O/bench_$M.log | cut -c1-140
done
