cd /root/repo
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/bert -o bert -- python3 bench.py --steps 10 --warmup 3 > gpurun_out/prof_bert.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/gpt -o gpt -- python3 bench.py --model gpt3-medium --steps 10 --warmup 3 > gpurun_out/prof_gpt.log 2>&1
