# round 5, call 16: implicit-GEMM conv with 256-row M tiles (FFK_CONV_BM=256) vs 128:
# conv numerics under the forced 256 tile, then the per-layer ResNet-50 bench both ways
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5g16; mkdir -p $O
FFK_CONV_BM=256 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_gpu.py > $O/tests256.txt 2>&1
rc=$?; tail -3 $O/tests256.txt; [ $rc -eq 0 ] || exit $rc
FFK_CONV_BM=128 timeout -k 10 400 python -u tools/bench_conv.py > $O/conv128.jsonl 2>&1 || { tail -5 $O/conv128.jsonl; exit 1; }
FFK_CONV_BM=256 timeout -k 10 400 python -u tools/bench_conv.py > $O/conv256.jsonl 2>&1 || { tail -5 $O/conv256.jsonl; exit 1; }
python - <<PY
import json
a=[json.loads(l) for l in open("$O/conv128.jsonl") if l.startswith("{")]
b=[json.loads(l) for l in open("$O/conv256.jsonl") if l.startswith("{")]
for x,y in zip(a,b):
    if x["bench"]!="conv": print(x, y); continue
    print(x["H"],x["C"],x["K"],x["R"],x["stride"],"x%d"%x["count"],"fwd",x["fwd_ms"],y["fwd_ms"],"dgrad",x["dgrad_ms"],y["dgrad_ms"],"wgrad",x["wgrad_ms"],"miopen",x["miopen_fwd_ms"],x["miopen_bwd_ms"])
PY
