# round 5, call 10: attention forward with 16-B output stores -- numerics
# (attention GPU tests) and same-process A/B
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5g10; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "attn or attention" tests/test_sequence_gpu.py > $O/tests.txt 2>&1
rc=$?; tail -3 $O/tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/attn_time.py --wide-ab > $O/attn_wide_ab.jsonl 2>&1 || { tail -20 $O/attn_wide_ab.jsonl; exit 1; }
grep shape $O/attn_wide_ab.jsonl
