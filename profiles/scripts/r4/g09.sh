# round 4, call 9: the whole GPU test tier, smoke(), and the 1-GPU benches of
# the four configs (same box)
set -o pipefail
mkdir -p gpurun_out/r4g09
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/r4g09/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/r4g09/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/r4g09/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4g09/smoke.log 2>&1 \
    || { tail -20 gpurun_out/r4g09/smoke.log; exit 1; }
tail -2 gpurun_out/r4g09/smoke.log
