# round 5, call 15: ping-pong A B^T kernel with A triple-buffered (prefetch distance 2, y2 / y6)
# vs split DMA (y1 / y5) vs hipBLASLt on the BERT dX shapes
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5g15; mkdir -p $O
timeout -k 10 300 python -u tools/gemm_ab.py --only dx --cands blaslt,w,y --rounds 3 --iters 10 > $O/ab.jsonl 2>&1 || { tail -20 $O/ab.jsonl; exit 1; }
python -c "
import json
for l in open('$O/ab.jsonl'):
    try: d=json.loads(l)
    except Exception: continue
    print(d['case'], {k:(d[k], d[k+'_err']) for k in d if k in ('blaslt','w1','y1','y2','y5','y6')})"
