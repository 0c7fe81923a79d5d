# round 5, call 24: conv K-tile fragments all requested before the first MFMA (sched_barrier):
# numerics, per-layer bench vs r5g22, ResNet-50 step
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5g24; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_gpu.py > $O/tests.txt 2>&1
rc=$?; tail -3 $O/tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/bench_conv.py > $O/conv.jsonl 2>&1 || { tail -5 $O/conv.jsonl; exit 1; }
python - <<PY
import json
a=[json.loads(l) for l in open("$R/profiles/r5/conv_r5_g22_stats.jsonl") if l.startswith("{")]
b=[json.loads(l) for l in open("$O/conv.jsonl") if l.startswith("{")]
for x,y in zip(a,b):
    if x["bench"]!="conv": print(x, y); continue
    print(x["H"],x["C"],x["K"],x["R"],x["stride"],"x%d"%x["count"],"fwd",x["fwd_ms"],y["fwd_ms"],"dgrad",x["dgrad_ms"],y["dgrad_ms"],"wgrad",x["wgrad_ms"],y["wgrad_ms"])
PY
timeout -k 10 300 python bench.py --model resnet50 --steps 20 --warmup 5 > $O/bench_rn.jsonl 2>&1 || { tail -20 $O/bench_rn.jsonl; exit 1; }
tail -1 $O/bench_rn.jsonl | cut -c1-200
