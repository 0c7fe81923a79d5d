# round 5, call 14: ping-pong A B^T kernel timing ablations (y7 no DMA in the loop,
# y11 no fragment reads, y15 neither) on dx_ffn1 / dx_head
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5g14; mkdir -p $O
timeout -k 10 300 python -u tools/gemm_ab.py --only dx --shapes dx_ffn1,dx_head,dx_qkv --cands blaslt,y --rounds 3 --iters 10 > $O/ab_abl.jsonl 2>&1 || { tail -20 $O/ab_abl.jsonl; exit 1; }
python -c "
import json
for l in open('$O/ab_abl.jsonl'):
    try: d=json.loads(l)
    except Exception: continue
    print(d['case'], {k:d[k] for k in d if k in ('blaslt','y0','y1','y2','y3','y7','y11','y15')})"
