# A/B of graph-timed autotuning (FF_AUTOTUNE_GRAPH) on BERT-large and ResNet-50, same box.
set -o pipefail
bash tools/ab_env.sh FF_AUTOTUNE_GRAPH "--model resnet50 --steps 20 --warmup 5" ab_autotune_graph_resnet || exit $?
bash tools/ab_env.sh FF_AUTOTUNE_GRAPH "--steps 10 --warmup 3" ab_autotune_graph_bert
