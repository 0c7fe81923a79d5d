# round 5, call 26: 32-deep register-staged ping-pong A B^T GEMM (variant 12, z1): numerics,
# then the BERT dX shapes against hipBLASLt / w / y
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5g26; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "gemmpp or pingpong8" > $O/tests.txt 2>&1
rc=$?; tail -3 $O/tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/gemm_ab.py --only dx --cands blaslt,w,y,z --rounds 3 --iters 10 > $O/ab.jsonl 2>&1 || { tail -20 $O/ab.jsonl; exit 1; }
python -c "
import json
for l in open('$O/ab.jsonl'):
    try: d=json.loads(l)
    except Exception: continue
    print(d['case'], {k:(d[k], d[k+'_err']) for k in d if k in ('blaslt','w1','y6','z1')})"
timeout -k 10 300 python -u tools/gemm_ab.py --only dx --cands blaslt,y,z --rounds 3 --iters 10 --beta 1 --shapes dx_qkv,dx_ffn2 > $O/ab_beta.jsonl 2>&1 || { tail -20 $O/ab_beta.jsonl; exit 1; }
python -c "
import json
for l in open('$O/ab_beta.jsonl'):
    try: d=json.loads(l)
    except Exception: continue
    print('beta1', d['case'], {k:(d[k], d[k+'_err']) for k in d if k in ('blaslt','y6','z1')})"
