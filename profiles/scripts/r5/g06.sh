# round 5, call 6: narrow-Linear / fused MSE kernels (tests), BN kernels with
# U rows per iteration (tests + bandwidth A/B + ResNet-50 A/B), DLRM bench
# and kernel trace (which torch element-wise / library kernels remain)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5g06; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_narrow_gpu.py tests/test_conv_gpu.py tests/test_runtime_c_gpu.py > $O/tests.txt 2>&1
rc=$?; tail -15 $O/tests.txt; [ $rc -eq 0 ] || exit $rc
for U in 1 2 4; do
  FFK_BN_UNROLL=$U timeout -k 10 200 python tools/bench_bn.py > $O/bench_bn_u$U.jsonl 2>&1 || { tail -5 $O/bench_bn_u$U.jsonl; exit 1; }
  echo "U=$U"; cut -c1-420 $O/bench_bn_u$U.jsonl
done
for U in 1 4; do
  FFK_BN_UNROLL=$U timeout -k 10 300 python bench.py --model resnet50 --steps 20 --warmup 5 > $O/bench_rn50_u$U.log 2>&1 || { tail -20 $O/bench_rn50_u$U.log; exit 1; }
  echo "rn50 U=$U"; tail -1 $O/bench_rn50_u$U.log | cut -c1-200
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python3 $R/bench.py --model dlrm --steps 50 --warmup 10 > $O/bench_dlrm.log 2>&1 || { tail -20 $O/bench_dlrm.log; exit 1; }
tail -1 $O/bench_dlrm.log | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_dlrm -o dl -- \
    python3 $R/bench.py --model dlrm --steps 5 --warmup 3 --graph 0 > $O/prof_dlrm.log 2>&1 || { tail -20 $O/prof_dlrm.log; exit 1; }
DB=$(find $O/prof_dlrm -name "dl_results.db" | head -n 1)
[ -n "$DB" ] && python3 $R/tools/prof_summary.py $DB --steps 5 --top 40 > $O/dlrm_kernels.txt
head -45 $O/dlrm_kernels.txt
