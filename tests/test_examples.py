"""Every example program runs end to end (small sample counts, CPU) and
prints the reference's THROUGHPUT line."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# every PyTorch-frontend example (reference: examples/python/pytorch/*.py);
# the *_torch.py / export_* scripts only write a .ff file
EXAMPLES = sorted(f"pytorch/{f}" for f in os.listdir(os.path.join(ROOT, "examples", "pytorch"))
                  if f.endswith(".py") and not f.startswith("_"))
# every ONNX example (reference: examples/python/onnx/*.py); *_pt / *_keras export
EXAMPLES += sorted(f"onnx/{f}" for f in os.listdir(os.path.join(ROOT, "examples", "onnx"))
                   if f.endswith(".py") and not f.startswith("_") and f != "accuracy.py")
EXAMPLES += ["pytorch/mt5/mt5_ff.py", "pytorch/mt5/mt5_torch.py", "keras/candle_uno/candle_uno.py"]
EXPORT_ONLY = {"pytorch/cifar10_cnn_torch.py", "pytorch/resnet_torch.py", "pytorch/torch_vision_torch.py",
               "pytorch/export_regnet_fx.py"} | {e for e in EXAMPLES if e.startswith("onnx/") and
                                                 (e.endswith("_pt.py") or e.endswith("_keras.py"))}
# every native example (reference: examples/python/native/*.py)
EXAMPLES += sorted(f"native/{f}" for f in os.listdir(os.path.join(ROOT, "examples", "native"))
                   if f.endswith(".py") and not f.startswith("_") and f != "accuracy.py")
# the 229 / 299-pixel CNNs run a couple of tiny batches on the CPU
HEAVY = {"native/alexnet.py", "native/inception.py", "native/resnet.py", "keras/func_cifar10_alexnet.py",
         "pytorch/resnet.py", "pytorch/regnet.py", "pytorch/torch_vision.py", "pytorch/resnet152_training.py",
         "onnx/alexnet.py", "onnx/resnet.py"}
# every keras example (reference: examples/python/keras/*.py)
KERAS = sorted(f for f in os.listdir(os.path.join(ROOT, "examples", "keras"))
               if f.endswith(".py") and not f.startswith("_") and f != "accuracy.py")
EXAMPLES += [f"keras/{f}" for f in KERAS]


@pytest.mark.parametrize("script", EXAMPLES)
def test_example_runs(script, tmp_path):
    heavy = script in HEAVY
    env = dict(os.environ, FF_EXAMPLE_SAMPLES="4" if heavy else "128", HIP_VISIBLE_DEVICES="", CUDA_VISIBLE_DEVICES="",
               FF_EXAMPLE_DIR=str(tmp_path))
    r = subprocess.run([sys.executable, os.path.join(ROOT, "examples", script), "-b", "2" if heavy else "32"],
                       cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    if script in EXPORT_ONLY:
        assert any(f.endswith((".ff", ".onnx")) for f in os.listdir(tmp_path)), r.stdout[-2000:]
    else:
        assert "THROUGHPUT" in r.stdout, r.stdout[-2000:]


def test_model_zoo_runner():
    env = dict(os.environ, HIP_VISIBLE_DEVICES="", CUDA_VISIBLE_DEVICES="")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "examples", "train.py"), "--model", "mlp_unify",
                        "--steps", "2", "--warmup", "1", "--config", '{"batch_size": 16, "input_dim": 64, "hidden_dims": [64, 64]}'],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "THROUGHPUT" in r.stdout
