"""Every example program runs end to end (small sample counts, CPU) and
prints the reference's THROUGHPUT line."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXAMPLES = ["pytorch/mnist_mlp_torch.py"]
# every native example (reference: examples/python/native/*.py)
EXAMPLES += sorted(f"native/{f}" for f in os.listdir(os.path.join(ROOT, "examples", "native"))
                   if f.endswith(".py") and not f.startswith("_") and f != "accuracy.py")
# the 229 / 299-pixel CNNs run a couple of tiny batches on the CPU
HEAVY = {"native/alexnet.py", "native/inception.py", "native/resnet.py", "keras/func_cifar10_alexnet.py"}
# every keras example (reference: examples/python/keras/*.py)
KERAS = sorted(f for f in os.listdir(os.path.join(ROOT, "examples", "keras"))
               if f.endswith(".py") and not f.startswith("_") and f != "accuracy.py")
EXAMPLES += [f"keras/{f}" for f in KERAS]


@pytest.mark.parametrize("script", EXAMPLES)
def test_example_runs(script):
    heavy = script in HEAVY
    env = dict(os.environ, FF_EXAMPLE_SAMPLES="4" if heavy else "128", HIP_VISIBLE_DEVICES="", CUDA_VISIBLE_DEVICES="")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "examples", script), "-b", "2" if heavy else "32"],
                       cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "THROUGHPUT" in r.stdout, r.stdout[-2000:]


def test_model_zoo_runner():
    env = dict(os.environ, HIP_VISIBLE_DEVICES="", CUDA_VISIBLE_DEVICES="")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "examples", "train.py"), "--model", "mlp_unify",
                        "--steps", "2", "--warmup", "1", "--config", '{"batch_size": 16, "input_dim": 64, "hidden_dims": [64, 64]}'],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "THROUGHPUT" in r.stdout
