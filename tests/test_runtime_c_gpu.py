"""The legacy C API (csrc/ffi/flexflow_runtime_c.h) on the GPU backing
(csrc/ffdev/device_exec.cpp): the C test program passes with its MLP and its
conv / batch-norm / pooling CNN on the GPU, and three Adam steps of a tanh /
sigmoid MLP under MSE and of a conv / BN / max+avg-pool CNN under
cross-entropy, and of a 2-layer BERT-style encoder (embedding, multi-head
attention, layer norms, dropout, split / concat, batch matmul) give the same
weights on the GPU as on the CPU backing (fp32 reference of the same ops)."""
import os
import re
import subprocess

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "bin", "ffc-runtime-c-test")


def _run(**env):
    e = dict(os.environ)
    e.update(env)
    r = subprocess.run([EXE], capture_output=True, text=True, timeout=300, env=e, cwd=ROOT)
    assert r.returncode == 0 and "PASSED (0 failures)" in r.stdout, r.stdout[-3000:] + r.stderr[-2000:]
    m = re.search(r"parity device (\S+).* w2_sum (\S+) w2_abs (\S+) w2_0 (\S+)", r.stdout)
    c = re.search(r"parity_cnn device (\S+).* w_sum (\S+) w_abs (\S+) w_0 (\S+)", r.stdout)
    b = re.search(r"parity_bert device (\S+).* emb_sum (\S+) attn_sum (\S+) attn_abs (\S+) attn_0 (\S+)", r.stdout)
    assert m and c and b, r.stdout
    return (r.stdout, m.group(1), [float(m.group(i)) for i in (2, 3, 4)] + [float(c.group(i)) for i in (2, 3, 4)],
            c.group(1), b.group(1), [float(b.group(i)) for i in (2, 3, 4, 5)])


def test_c_api_trains_on_gpu_and_matches_cpu():
    if not os.path.exists(EXE):
        pytest.skip("C API test program not built")
    out_gpu, dev_gpu, vals_gpu, cnn_gpu, bert_gpu, bvals_gpu = _run()
    out_cpu, dev_cpu, vals_cpu, cnn_cpu, bert_cpu, bvals_cpu = _run(FF_C_API_DEVICE="cpu")
    assert "device gpu:" in out_gpu, out_gpu[:2000]     # the MLP compiled onto the GPU backing
    assert "cnn device gpu:" in out_gpu, out_gpu[:3000]  # conv / batch norm / pooling too
    assert dev_gpu.startswith("gpu:") and dev_cpu == "cpu", (dev_gpu, dev_cpu)
    assert cnn_gpu.startswith("gpu:") and cnn_cpu == "cpu", (cnn_gpu, cnn_cpu)
    for g, c in zip(vals_gpu, vals_cpu):
        assert abs(g - c) <= 1e-4 * max(1.0, abs(c)), (vals_gpu, vals_cpu)
    # the 2-layer BERT (embedding, attention, layer norm, dropout, split /
    # concat, batch matmul) trains on the GPU backing and matches the CPU one
    assert bert_gpu.startswith("gpu:") and bert_cpu == "cpu", (bert_gpu, bert_cpu, out_gpu[-3000:])
    for g, c in zip(bvals_gpu, bvals_cpu):
        assert abs(g - c) <= 1e-4 * max(1.0, abs(c)), (bvals_gpu, bvals_cpu)
