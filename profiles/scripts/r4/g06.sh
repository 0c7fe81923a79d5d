# round 4, call 6: in-situ per-operator costs (timed inside each bench
# config's own 1-GPU data-parallel training step, fusions included) for the
# simulator calibration (tools/search_report.py --calibrate)
set -o pipefail
mkdir -p gpurun_out/calib
export TMPDIR=/tmp
for M in ${MODELS:-bert-large dlrm gpt3-medium resnet50}; do
  timeout -k 10 300 python -u tools/profile_ops.py --model $M --world 1 --in-situ \
      --out gpurun_out/calib/op_costs_${M}_insitu_w1.json > gpurun_out/calib/insitu_$M.log 2>&1 \
      || { tail -20 gpurun_out/calib/insitu_$M.log; exit 1; }
  tail -1 gpurun_out/calib/insitu_$M.log
done
