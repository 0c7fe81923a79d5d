#!/bin/bash
# round 5, call 42: final HEAD GPU tier + smoke
set -o pipefail
O=gpurun_out/r5g42; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.txt 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1
