# round 5, call 3: where each hand-written GEMM stands vs hipBLASLt at the
# BERT-large b64 shapes (forward NN + input-gradient NT): gemmt kk (w),
# ping-pong (r), eight-wave NT (n), gemmq (q)
set -o pipefail
O=gpurun_out/r5g03; mkdir -p $O
timeout -k 10 500 python -u tools/gemm_ab.py --only fwd,dx --cands blaslt,w,r,n,q --rounds 3 --iters 10 > $O/ab.jsonl 2>&1 || { tail -20 $O/ab.jsonl; exit 1; }
python - <<'PY'
import json
for l in open("gpurun_out/r5g03/ab.jsonl"):
    if not l.startswith("{"): continue
    d = json.loads(l)
    ks = [k for k in d if k.endswith("_TF")]
    print(d["case"], " ".join(f"{k[:-3]}:{d[k]}" for k in ks), "best", d["best"])
PY
