"""PyTorch -> FlexFlow: trace an nn.Module with torch.fx, write the .ff IR,
rebuild it in an FFModel, copy the weights and train
(reference: examples/python/pytorch/mnist_mlp_torch.py + mnist_mlp.py)."""
import os
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import numpy as np  # noqa: E402
import torch.nn as nn  # noqa: E402

from flexflow.core import DataType, FFConfig, FFModel, LossType, MetricsType, SGDOptimizer  # noqa: E402
from flexflow.keras.datasets import mnist  # noqa: E402
from flexflow.torch.fx import torch_to_flexflow  # noqa: E402
from flexflow.torch.model import PyTorchModel  # noqa: E402


class MLP(nn.Module):
    def __init__(self):
        super().__init__()
        self.linear1 = nn.Linear(784, 512)
        self.linear2 = nn.Linear(512, 512)
        self.linear3 = nn.Linear(512, 10)
        self.relu = nn.ReLU()
        self.softmax = nn.Softmax(dim=-1)

    def forward(self, x):
        x = self.relu(self.linear1(x))
        x = self.relu(self.linear2(x))
        return self.softmax(self.linear3(x))


def top_level_task():
    path = os.path.join(tempfile.mkdtemp(), "mlp.ff")
    torch_to_flexflow(MLP(), path)          # the .ff text IR (one node per line)
    ffconfig = FFConfig()
    ffconfig.parse_args()
    m = FFModel(ffconfig)
    x = m.create_tensor([ffconfig.batch_size, 784], DataType.DT_FLOAT)
    PyTorchModel.file_to_ff(path, m, [x])
    m.optimizer = SGDOptimizer(m, 0.01)
    m.compile(loss_type=LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY, metrics=[MetricsType.METRICS_ACCURACY])
    n = int(os.environ.get("FF_EXAMPLE_SAMPLES", 60000))
    (xt, yt), _ = mnist.load_data(num_samples=n)
    xt = xt.reshape(len(xt), 784).astype("float32") / 255
    m.fit(x=xt, y=yt.astype("int32").reshape(-1, 1), epochs=ffconfig.epochs)


if __name__ == "__main__":
    top_level_task()
