# round 4, call 2: distributed-path rehearsal of the BERT-large bench at world 1
# over RCCL (graph segments + bucketed all-reduce), then the autotune stall repro
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
FF_DIST_WORLD1=1 timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_bert_world1_rccl.log 2>&1 && \
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_bert_plain.log 2>&1 && \
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/stall_prof -o run -- python tools/autotune_stall_repro.py child eager 256 1024 256 > gpurun_out/stall_prof.log 2>&1 && \
timeout -k 10 600 python -u tools/autotune_stall_repro.py > gpurun_out/stall_repro.log 2>&1
