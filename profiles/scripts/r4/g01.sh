# round 4, call 1: RCCL world-1 test, benches with the queued autotune clock,
# then the autotuner graph-clock stall diagnostic (last: it may hang)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_rccl_gpu.py > gpurun_out/rccl_test.log 2>&1 && \
timeout -k 10 400 python -u bench.py --model dlrm --steps 20 --warmup 5 > gpurun_out/bench_dlrm.log 2>&1 && \
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_bert.log 2>&1 && \
FF_AUTOTUNE_GRAPH=1 FF_AUTOTUNE_GRAPH_SYNC=1 FF_AUTOTUNE_TRACE=1 timeout -k 10 150 python -u -X faulthandler -c "import faulthandler; faulthandler.dump_traceback_later(100, exit=True); import __graft_entry__ as g; g.smoke(); print('SMOKE OK sync=1')" > gpurun_out/stall_sync1.log 2>&1 && \
FF_AUTOTUNE_GRAPH=1 FF_AUTOTUNE_GRAPH_SYNC=0 FF_AUTOTUNE_TRACE=1 timeout -k 10 150 python -u -X faulthandler -c "import faulthandler; faulthandler.dump_traceback_later(100, exit=True); import __graft_entry__ as g; g.smoke(); print('SMOKE OK sync=0')" > gpurun_out/stall_sync0.log 2>&1
