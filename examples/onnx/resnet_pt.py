"""Export ResNet-18 from PyTorch to resnet18.onnx (reference:
examples/python/onnx/resnet_pt.py; the network definition is shared with
examples/pytorch/resnet_torch.py)."""
import os
import sys

import torch
from _common import onnx_path

from flexflow.onnx.model import ONNXModel, export_torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "pytorch"))
from resnet_torch import resnet18  # noqa: E402


def export(path=None):
    path = path or onnx_path("resnet18.onnx")
    export_torch(resnet18(num_classes=10), torch.randn(2, 3, 224, 224), path, export_params=False)
    return path


if __name__ == "__main__":
    g = ONNXModel(export()).graph
    for node in g.nodes:
        print(node.op_type, node.inputs, node.outputs)
    for name, dims, _ in g.inputs:
        print(name, dims)
