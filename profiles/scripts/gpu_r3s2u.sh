# Final check after making graph-timed autotuning opt-in: full GPU tests, smoke, BERT / DLRM / GPT / ResNet benches.
set -o pipefail
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/u_tests.log 2>&1 || exit $?
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > gpurun_out/u_smoke.log 2>&1 || exit $?
timeout -k 10 200 python -u bench.py > gpurun_out/u_bert_default.log 2>&1 || exit $?
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > gpurun_out/u_bert.log 2>&1 || exit $?
timeout -k 10 200 python -u bench.py --model dlrm --steps 20 --warmup 5 > gpurun_out/u_dlrm.log 2>&1 || exit $?
timeout -k 10 200 python -u bench.py --model gpt3-medium --steps 10 --warmup 3 > gpurun_out/u_gpt.log 2>&1 || exit $?
timeout -k 10 200 python -u bench.py --model resnet50 --steps 20 --warmup 5 > gpurun_out/u_resnet.log 2>&1
