# round 5, call 22: conv BN statistics reduced from the stored C tile (per-thread column sums,
# 2-3 shuffles, 4-wave LDS sum, one partial row per tile): numerics, 1x1 probe, per-layer bench
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5g22; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_gpu.py tests/test_executor_gpu.py > $O/tests.txt 2>&1
rc=$?; tail -3 $O/tests.txt; [ $rc -eq 0 ] || exit $rc
cd $R/tools && timeout -k 10 300 python -u conv1x1_probe.py > $O/probe.jsonl 2>&1 || { tail -5 $O/probe.jsonl; exit 1; }
cat $O/probe.jsonl
cd $R && timeout -k 10 400 python -u tools/bench_conv.py > $O/conv.jsonl 2>&1 || { tail -5 $O/conv.jsonl; exit 1; }
tail -1 $O/conv.jsonl
timeout -k 10 300 python bench.py --model resnet50 --steps 20 --warmup 5 > $O/bench_rn.jsonl 2>&1 || { tail -20 $O/bench_rn.jsonl; exit 1; }
tail -1 $O/bench_rn.jsonl | cut -c1-200
