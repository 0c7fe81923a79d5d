# Full GPU validation + the four 1-GPU benches (results under gpurun_out/).
set -o pipefail
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_bert.log 2>&1 && \
timeout -k 10 400 python -u bench.py --model resnet50 --steps 20 --warmup 5 > gpurun_out/bench_resnet.log 2>&1 && \
timeout -k 10 400 python -u bench.py --model gpt3-medium --steps 10 --warmup 3 > gpurun_out/bench_gpt.log 2>&1 && \
timeout -k 10 400 python -u bench.py --model dlrm --steps 20 --warmup 5 > gpurun_out/bench_dlrm.log 2>&1
