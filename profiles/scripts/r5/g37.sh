#!/bin/bash
# HEAD verification: full GPU tier, smoke, default bench, ResNet-50 bench
set -o pipefail
mkdir -p gpurun_out/r5g37
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5g37/tests.txt 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5g37/smoke.txt 2>&1 &&
timeout -k 10 400 python bench.py > gpurun_out/r5g37/bench_default.json 2> gpurun_out/r5g37/bench.err &&
timeout -k 10 300 python bench.py --model resnet50 --steps 20 --warmup 5 > gpurun_out/r5g37/rn50.json 2>> gpurun_out/r5g37/bench.err
