# BERT-large kernel profile + GEMM autotune report at the 64/GPU default; 2-rank gloo rehearsal.
set -o pipefail
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
FF_GEMM_REPORT=1 timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/bench_bert_rep.log 2> gpurun_out/gemm_report_b64.txt || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/bert64 -o bert -- python3 bench.py --steps 10 --warmup 3 > gpurun_out/prof_bert64.log 2>&1 || exit $?
bash tools/rehearse_multi.sh 2 bert-large > gpurun_out/rehearse2.log 2>&1
