# round 4, call 29: final GPU tier + smoke on the tree as committed
set -o pipefail
O=gpurun_out/r4g29; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.txt 2>&1 \
  || { tail -30 $O/gpu_tests.txt; exit 1; }
tail -1 $O/gpu_tests.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || exit 1
tail -1 $O/bench.log | cut -c1-160
