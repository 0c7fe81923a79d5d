# round 5, call 30: ping-pong GEMM with 2 / 3 / 4 LDS-DMA pieces per wave moved into the compute
# half (y22 / y30 / y38) vs mode 6 (y6), w and hipBLASLt on the BERT dX shapes
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5g30; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "gemmpp or pingpong8" > $O/tests.txt 2>&1
rc=$?; tail -3 $O/tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/gemm_ab.py --only dx --cands blaslt,w,y --rounds 3 --iters 10 > $O/ab.jsonl 2>&1 || { tail -20 $O/ab.jsonl; exit 1; }
python -c "
import json
for l in open('$O/ab.jsonl'):
    try: d=json.loads(l)
    except Exception: continue
    print(d['case'], {k:d[k] for k in d if k in ('blaslt','w1','y6','y22','y30','y38')})"
