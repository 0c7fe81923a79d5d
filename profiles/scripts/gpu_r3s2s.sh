# End-of-session evidence: full GPU tests, smoke, DLRM kernel profile.
set -o pipefail
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/final_gpu_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > gpurun_out/final_smoke.log 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/dlrm3 -o dlrm -- python3 bench.py --model dlrm --steps 20 --warmup 5 > gpurun_out/prof_dlrm3.log 2>&1
