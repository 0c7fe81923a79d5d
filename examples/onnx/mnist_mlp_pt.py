"""Export the MNIST MLP from PyTorch to mnist_mlp_pt.onnx (reference:
examples/python/onnx/mnist_mlp_pt.py; torch.onnx.export's role is played by
flexflow.onnx.export_torch since the onnx package is not installed)."""
import torch
import torch.nn as nn
from _common import onnx_path

from flexflow.onnx.model import ONNXModel, export_torch


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


def export(path=None):
    path = path or onnx_path("mnist_mlp_pt.onnx")
    export_torch(MLP(), torch.randn(100, 784), path, export_params=False)
    return path


if __name__ == "__main__":
    p = export()
    for node in ONNXModel(p).graph.nodes:
        print(node.op_type, node.inputs, node.outputs)
