# DLRM kernel profile after the native row-sparse SGD.
set -o pipefail
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/dlrm2 -o dlrm -- python3 bench.py --model dlrm --steps 20 --warmup 5 > gpurun_out/prof_dlrm2.log 2>&1
