# round 4, call 10: bisect the NaN of test_segmented_graph_data_parallel
# (bert_tiny, graphed DP step over gloo) across this round's kernel switches
set -o pipefail
mkdir -p gpurun_out/r4g10
export TMPDIR=/tmp
T="tests/test_segmented_graph_gpu.py::test_segmented_graph_data_parallel"
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 200 python -u -m pytest "$T" -x -q --timeout 150 --timeout-method thread \
      > gpurun_out/r4g10/$name.log 2>&1
  echo "$name rc=$? $(tail -1 gpurun_out/r4g10/$name.log)"
}
run default
run emb_small_off FFK_EMB_SMALL=0
run fused_delta_off FFK_ATTN_BWD_FUSED_DELTA=0
run both_off FFK_EMB_SMALL=0 FFK_ATTN_BWD_FUSED_DELTA=0
