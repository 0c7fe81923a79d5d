# round 5, call 2: ResNeXt-50 (grouped convs on igemm32) bench + kernel trace
# (no MIOpen / library conv kernels), an fp32 ResNet-50 step, BERT baseline
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5g02; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 python3 $R/bench.py --model resnext50 --steps 10 --warmup 3 > $O/bench_resnext50.log 2>&1 || { tail -20 $O/bench_resnext50.log; exit 1; }
tail -1 $O/bench_resnext50.log | cut -c1-300
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_rx -o rx -- \
    python3 $R/bench.py --model resnext50 --steps 3 --warmup 2 > $O/prof_rx.log 2>&1 || { tail -20 $O/prof_rx.log; exit 1; }
DB=$(find $O/prof_rx -name "rx_results.db" | head -n 1)
[ -n "$DB" ] && python3 $R/tools/prof_summary.py $DB --steps 3 --top 40 > $O/resnext50_kernels.txt
head -45 $O/resnext50_kernels.txt
timeout -k 10 400 python3 $R/bench.py --model resnet50 --dtype float32 --batch-per-gpu 64 --steps 5 --warmup 2 > $O/bench_resnet50_fp32.log 2>&1 || { tail -20 $O/bench_resnet50_fp32.log; exit 1; }
tail -1 $O/bench_resnet50_fp32.log | cut -c1-300
timeout -k 10 400 python3 $R/bench.py --steps 20 --warmup 5 > $O/bench_bert.log 2>&1 || exit 1
tail -1 $O/bench_bert.log | cut -c1-250
