# round 4, call 4: simulator calibration inputs on one box — per-op cost
# tables of the data-parallel pieces at each bench config's per-GPU batch,
# and the measured 1-GPU step time of the same config (bench.py --strategy dp)
set -o pipefail
mkdir -p gpurun_out/calib
for M in ${MODELS:-bert-large gpt3-medium resnet50 dlrm}; do
  timeout -k 10 420 python -u tools/profile_ops.py --model $M --world 1 \
      --out gpurun_out/calib/op_costs_${M}_w1.json > gpurun_out/calib/prof_$M.log 2>&1 || exit 1
  timeout -k 10 300 python -u bench.py --model $M --strategy dp --no-dp-compare --steps 10 --warmup 3 \
      > gpurun_out/calib/bench_$M.json 2> gpurun_out/calib/bench_$M.err || exit 1
  echo "done $M"
done
