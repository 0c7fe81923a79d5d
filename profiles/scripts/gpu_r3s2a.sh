# Per-GPU batch sweep for the BERT-large / GPT-3 medium benches (288 GB HBM leaves room).
set -o pipefail
for b in 32 48 64; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --batch-per-gpu $b > gpurun_out/bs_bert_$b.log 2>&1 || exit $?
done
for b in 8 16; do
  timeout -k 10 300 python -u bench.py --model gpt3-medium --steps 10 --warmup 3 --batch-per-gpu $b > gpurun_out/bs_gpt_$b.log 2>&1 || exit $?
done
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/gpt -o gpt -- python3 bench.py --model gpt3-medium --steps 10 --warmup 3 > gpurun_out/prof_gpt.log 2>&1
