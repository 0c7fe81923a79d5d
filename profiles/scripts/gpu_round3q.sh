set -o pipefail
FF_GEMM_REPORT=1 timeout -k 10 400 python -u bench.py --model gpt3-medium --steps 10 --warmup 3 > gpurun_out/bench_gpt.log 2> gpurun_out/bench_gpt_report.txt && \
cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_gpt -o gpt -- python3 $GRAFT_REPO_ROOT/bench.py --model gpt3-medium --steps 3 --warmup 2 > $GRAFT_REPO_ROOT/gpurun_out/prof_gpt.log 2>&1
