# round 5, call 8: zero-fill kernel test; DLRM and ResNet-50 kernel traces with
# the native-preferring GEMM autotuner (which library / torch kernels remain)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5g08; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_narrow_gpu.py tests/test_executor_gpu.py tests/test_conv_gpu.py tests/test_kernels_gpu.py > $O/tests.txt 2>&1
rc=$?; tail -3 $O/tests.txt; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python3 $R/bench.py --model dlrm --steps 50 --warmup 10 > $O/bench_dlrm.jsonl 2>&1 || { tail -20 $O/bench_dlrm.jsonl; exit 1; }
tail -1 $O/bench_dlrm.jsonl | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_dlrm -o dl -- \
    python3 $R/bench.py --model dlrm --steps 5 --warmup 3 --graph 0 > $O/prof_dlrm.log 2>&1 || { tail -20 $O/prof_dlrm.log; exit 1; }
DB=$(find $O/prof_dlrm -name "dl_results.db" | head -n 1)
[ -n "$DB" ] && python3 $R/tools/prof_summary.py $DB --steps 5 --top 30 > $O/dlrm_kernels.txt
head -34 $O/dlrm_kernels.txt
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_rn -o rn -- \
    python3 $R/bench.py --model resnet50 --steps 5 --warmup 3 > $O/prof_rn.log 2>&1 || { tail -20 $O/prof_rn.log; exit 1; }
DB=$(find $O/prof_rn -name "rn_results.db" | head -n 1)
[ -n "$DB" ] && python3 $R/tools/prof_summary.py $DB --steps 5 --top 40 > $O/rn50_kernels.txt
head -44 $O/rn50_kernels.txt
cd $R
FF_AUTOTUNE_REPORT=$O/autotune_bert.txt timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_bert.jsonl 2>&1 || { tail -20 $O/bench_bert.jsonl; exit 1; }
tail -1 $O/bench_bert.jsonl | cut -c1-700
cat $O/autotune_bert.txt
