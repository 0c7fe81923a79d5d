# round 4, call 21: GPU tier + smoke at HEAD, then per-kernel time of the
# BERT-large and GPT-3 medium bench steps with gemmt_kk_kernel (kernel trace,
# last 5 optimizer steps) and plain bench runs
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4g21; mkdir -p $O
cd $R && timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.txt 2>&1 \
  || { tail -30 $O/gpu_tests.txt; exit 1; }
tail -1 $O/gpu_tests.txt
cd $R && timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
cd /tmp && export TMPDIR=/tmp
for M in bert-large gpt3-medium; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_$M -o $M -- \
      python3 $R/bench.py --model $M --steps 5 --warmup 3 > $O/prof_$M.log 2>&1 \
      || { tail -20 $O/prof_$M.log; exit 1; }
  DB=$(ls $O/prof_$M/*/${M}_results.db 2>/dev/null | head -n 1 || true)
  [ -z "$DB" ] && DB=$(ls $O/prof_$M/${M}_results.db 2>/dev/null || true)
  [ -n "$DB" ] && python3 $R/tools/prof_summary.py $DB --steps 5 --top 40 > $O/${M}_kernels.txt
  rm -rf $O/prof_$M
done
for M in bert-large gpt3-medium; do
  timeout -k 10 400 python3 $R/bench.py --model $M --steps 20 --warmup 5 > $O/bench_$M.log 2>&1 || exit 1
  tail -1 $O/bench_$M.log | cut -c1-140
done
