# round 4, call 27: per-kernel time of the BERT-large and GPT-3 medium bench
# steps at HEAD (gemmt_kk_kernel on TN / NN / NT), kernel trace, last 5 steps
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4g27; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for M in bert-large gpt3-medium; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_$M -o $M -- \
      python3 $R/bench.py --model $M --steps 5 --warmup 3 > $O/prof_$M.log 2>&1 \
      || { tail -20 $O/prof_$M.log; exit 1; }
  DB=$(ls $O/prof_$M/*/${M}_results.db 2>/dev/null | head -n 1 || true)
  [ -z "$DB" ] && DB=$(ls $O/prof_$M/${M}_results.db 2>/dev/null || true)
  [ -n "$DB" ] && python3 $R/tools/prof_summary.py $DB --steps 5 --top 40 > $O/${M}_kernels.txt
  rm -rf $O/prof_$M
  head -12 $O/${M}_kernels.txt | cut -c1-110
done
