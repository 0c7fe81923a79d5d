# DLRM kernel profile at the default batch (1024/GPU).
set -o pipefail
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/dlrm -o dlrm -- python3 bench.py --model dlrm --steps 20 --warmup 5 > gpurun_out/prof_dlrm.log 2>&1
