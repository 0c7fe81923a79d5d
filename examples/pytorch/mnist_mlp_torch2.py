"""nn.Module -> FFModel in one step (PyTorchModel.torch_to_ff, no .ff file)
(reference: examples/python/pytorch/mnist_mlp_torch2.py)."""
import numpy as np
import torch.nn as nn
from _common import num_samples, report

from flexflow.core import DataType, FFConfig, FFModel, LossType, MetricsType, SGDOptimizer
from flexflow.keras.datasets import mnist
from flexflow.torch.model import PyTorchModel


class MLP(nn.Module):
    def __init__(self):
        super().__init__()
        self.linear1 = nn.Linear(784, 512)
        self.linear2 = nn.Linear(512, 512)
        self.linear3 = nn.Linear(512, 10)
        self.relu = nn.ReLU()
        self.softmax = nn.Softmax(dim=-1)

    def forward(self, x):
        y = self.relu(self.linear1(x))
        y = self.relu(self.linear2(y))
        return self.softmax(self.linear3(y))


def top_level_task():
    ffconfig = FFConfig()
    ffconfig.parse_args()
    m = FFModel(ffconfig)
    x = m.create_tensor([ffconfig.batch_size, 784], DataType.DT_FLOAT)
    PyTorchModel(MLP()).torch_to_ff(m, [x])
    m.optimizer = SGDOptimizer(m, 0.01)
    m.compile(loss_type=LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY,
              metrics=[MetricsType.METRICS_ACCURACY, MetricsType.METRICS_SPARSE_CATEGORICAL_CROSSENTROPY])
    n = num_samples(60000)
    (xt, yt), _ = mnist.load_data(num_samples=n)
    dl_x = m.create_data_loader(x, xt.reshape(n, 784).astype("float32") / 255)
    dl_y = m.create_data_loader(m.label_tensor, np.reshape(yt.astype("int32"), (n, 1)))
    m.init_layers()
    ts = ffconfig.get_current_time()
    m.fit(x=dl_x, y=dl_y, epochs=ffconfig.epochs)
    report(ffconfig, ts, n, ffconfig.epochs)


if __name__ == "__main__":
    print("mnist mlp")
    top_level_task()
