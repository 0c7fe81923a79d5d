# round 5, call 23: ResNet-50 kernel trace after the conv loader / stats work
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5g23; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_rn -o rn -- \
    python3 $R/bench.py --model resnet50 --steps 5 --warmup 3 > $O/prof_rn.log 2>&1 || { tail -20 $O/prof_rn.log; exit 1; }
DB=$(find $O/prof_rn -name "rn_results.db" | head -n 1)
[ -n "$DB" ] && python3 $R/tools/prof_summary.py $DB --steps 5 --top 40 > $O/rn50_kernels.txt
head -44 $O/rn50_kernels.txt
