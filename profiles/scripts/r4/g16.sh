# round 4, call 16: per-kernel time of the GPT-3 medium, ResNet-50 and DLRM
# bench steps (kernel trace, last 5 optimizer steps of each)
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r4g16
cd /tmp && export TMPDIR=/tmp
for M in gpt3-medium resnet50 dlrm; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r4g16/prof_$M -o $M -- \
      python3 $R/bench.py --model $M --steps 5 --warmup 3 > $R/gpurun_out/r4g16/prof_$M.log 2>&1 \
      || { tail -20 $R/gpurun_out/r4g16/prof_$M.log; exit 1; }
  tail -1 $R/gpurun_out/r4g16/prof_$M.log | cut -c1-160
  DB=$(ls $R/gpurun_out/r4g16/prof_$M/*/${M}_results.db 2>/dev/null | head -n 1 || true)
  [ -z "$DB" ] && DB=$(ls $R/gpurun_out/r4g16/prof_$M/${M}_results.db 2>/dev/null || true)
  [ -n "$DB" ] && python3 $R/tools/prof_summary.py $DB --steps 5 --top 40 > $R/gpurun_out/r4g16/${M}_kernels.txt
  rm -rf $R/gpurun_out/r4g16/prof_$M
done
echo done
