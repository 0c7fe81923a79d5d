# round 5, call 4: gemmt_kk register-staged (variant 10, "x") -- correctness
# (test_gemmp, tightened bounds) and the same-process A/B against the LDS-DMA
# form ("w") and hipBLASLt on the BERT-large b64 shapes
set -o pipefail
O=gpurun_out/r5g04; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "test_gemmp" > $O/tests.txt 2>&1
rc=$?; tail -3 $O/tests.txt
timeout -k 10 500 python -u tools/gemm_ab.py --only fwd,dx,dw --cands blaslt,w,x --rounds 3 --iters 10 > $O/ab.jsonl 2>&1 || { tail -20 $O/ab.jsonl; exit 1; }
python - <<'PY'
import json
for l in open("gpurun_out/r5g04/ab.jsonl"):
    if not l.startswith("{"): continue
    d = json.loads(l)
    ks = [k for k in d if k.endswith("_TF")]
    print(d["case"], " ".join(f"{k[:-3]}:{d[k]}" for k in ks), "best", d["best"], "err_x", d.get("x1_err", d.get("x4_err")))
PY
exit $rc
