"""Export the CIFAR-10 CNN from PyTorch to cifar10_cnn_pt.onnx (reference:
examples/python/onnx/cifar10_cnn_pt.py)."""
import torch
import torch.nn as nn
from _common import onnx_path

from flexflow.onnx.model import ONNXModel, export_torch


class CNN(nn.Module):
    def __init__(self):
        super().__init__()
        self.conv1 = nn.Conv2d(3, 32, 3, 1)
        self.conv2 = nn.Conv2d(32, 32, 3, 1)
        self.pool1 = nn.MaxPool2d(2, 2)
        self.conv3 = nn.Conv2d(32, 64, 3, 1)
        self.conv4 = nn.Conv2d(64, 64, 3, 1)
        self.pool2 = nn.MaxPool2d(2, 2)
        self.flat1 = nn.Flatten()
        self.linear1 = nn.Linear(1600, 512)
        self.linear2 = nn.Linear(512, 10)
        self.relu = nn.ReLU()
        self.softmax = nn.Softmax(dim=-1)

    def forward(self, x):
        y = self.pool1(self.relu(self.conv2(self.relu(self.conv1(x)))))
        y = self.pool2(self.relu(self.conv4(self.relu(self.conv3(y)))))
        y = self.relu(self.linear1(self.flat1(y)))
        return self.softmax(self.linear2(y))


def export(path=None):
    path = path or onnx_path("cifar10_cnn_pt.onnx")
    export_torch(CNN(), torch.randn(64, 3, 32, 32), path, export_params=False)
    return path


if __name__ == "__main__":
    for node in ONNXModel(export()).graph.nodes:
        print(node.op_type, node.inputs, node.outputs)
