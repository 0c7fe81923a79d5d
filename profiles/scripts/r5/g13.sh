# round 5, call 13: first run of the eight-wave ping-pong A B^T kernel (gemmpp.hip,
# variant 11, modes y0-y3) against hipBLASLt and the one-wave kernels on the BERT dX shapes
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5g13; mkdir -p $O
timeout -k 10 300 python -u tools/gemm_ab.py --only dx --cands blaslt,w,x,y --rounds 3 --iters 10 > $O/ab_dx.jsonl 2>&1 || { tail -20 $O/ab_dx.jsonl; exit 1; }
cat $O/ab_dx.jsonl | python -c "
import sys,json
for l in sys.stdin:
    try: d=json.loads(l)
    except Exception: print(l.strip()); continue
    print(d['case'], {k:(d[k],d.get(k+'_err')) for k in d if k in ('blaslt','w1','x1','y0','y1','y2','y3')}, d['best'])"
timeout -k 10 300 python -u tools/gemm_ab.py --only dx --cands blaslt,w,x,y --rounds 3 --iters 10 --beta 1 --shapes dx_qkv,dx_ffn2,dx_head > $O/ab_dx_beta.jsonl 2>&1 || { tail -20 $O/ab_dx_beta.jsonl; exit 1; }
cat $O/ab_dx_beta.jsonl | cut -c1-600
