# Per-GPU batch sweep, larger batches (288 GB HBM per GPU).
set -o pipefail
for b in 96 128; do
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --batch-per-gpu $b > gpurun_out/bs_bert_$b.log 2>&1 || exit $?
done
for b in 24 32; do
  timeout -k 10 300 python -u bench.py --model gpt3-medium --steps 10 --warmup 3 --batch-per-gpu $b > gpurun_out/bs_gpt_$b.log 2>&1 || exit $?
done
for b in 512; do
  timeout -k 10 300 python -u bench.py --model resnet50 --steps 10 --warmup 3 --batch-per-gpu $b > gpurun_out/bs_resnet_$b.log 2>&1 || exit $?
done
for b in 4096 16384; do
  timeout -k 10 300 python -u bench.py --model dlrm --steps 20 --warmup 5 --batch-per-gpu $b > gpurun_out/bs_dlrm_$b.log 2>&1 || exit $?
done
