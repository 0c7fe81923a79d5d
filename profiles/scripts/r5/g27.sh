# round 5, call 27: native replay of segmented distributed steps (csrc/runtime/replay.cpp):
# RCCL world-1 training parity (DP / ZeRO / PS / embedding, graphed and eager), then BERT-large
# over the RCCL path at world 1 with the native walker and with the Python one
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5g27; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_rccl_gpu.py > $O/tests.txt 2>&1
rc=$?; tail -3 $O/tests.txt; [ $rc -eq 0 ] || exit $rc
FF_DIST_WORLD1=1 timeout -k 10 400 python bench.py --steps 10 --warmup 3 > $O/bench_w1_native.jsonl 2> $O/bench_w1_native.err || { tail -30 $O/bench_w1_native.err; exit 1; }
tail -1 $O/bench_w1_native.jsonl | cut -c1-200; grep -o '"graph_segments[^]]*], "native_replay": [a-z]*' $O/bench_w1_native.jsonl
FF_NATIVE_REPLAY=0 FF_DIST_WORLD1=1 timeout -k 10 400 python bench.py --steps 10 --warmup 3 > $O/bench_w1_py.jsonl 2> $O/bench_w1_py.err || { tail -30 $O/bench_w1_py.err; exit 1; }
tail -1 $O/bench_w1_py.jsonl | cut -c1-200; grep -o '"graph_segments[^]]*], "native_replay": [a-z]*' $O/bench_w1_py.jsonl
