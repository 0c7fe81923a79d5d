# 4-rank gloo rehearsals on one GPU (ranks share cuda:0): DLRM (searched table sharding) and BERT-large (searched).
set -o pipefail
bash tools/rehearse_multi.sh 4 dlrm > gpurun_out/rehearse4_dlrm.log 2>&1 || exit $?
bash tools/rehearse_multi.sh 4 bert-large > gpurun_out/rehearse4_bert.log 2>&1
