set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -k "test_gemmp" -x -q --timeout 60 --timeout-method thread > gpurun_out/gemmp_tests.log 2>&1 && \
timeout -k 10 600 python -u tools/gemm_ab.py --rounds 3 --iters 10 --cands blaslt,t,v > gpurun_out/gemm_ab.jsonl 2> gpurun_out/gemm_ab.err && \
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_bert.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_bert -o bert -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 3 > $GRAFT_REPO_ROOT/gpurun_out/prof_bert.log 2>&1
