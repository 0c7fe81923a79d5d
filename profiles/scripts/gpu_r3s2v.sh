# DLRM kernel profile after the round-3 changes.
set -o pipefail
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/dlrm4 -o dlrm -- python3 bench.py --model dlrm --steps 20 --warmup 5 > gpurun_out/prof_dlrm4.log 2>&1
