#!/bin/bash
# round 6, call 18: what is live at the step peak beyond the forward's activations (CNNs: plan -12..-17 %)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6g18; mkdir -p $O
cd $R
for m in "resnet50 256" "inception_v3 64"; do
  PYTHONPATH=$R timeout -k 10 300 python3 -u tools/mem_audit.py $m --trace > $O/audit_${m%% *}.txt 2>&1 || { tail -20 $O/audit_${m%% *}.txt; exit 1; }
  grep "step_peak_new\|peak_site\|^{\"model" $O/audit_${m%% *}.txt | cut -c1-300
done
