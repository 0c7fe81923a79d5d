"""Export AlexNet (the reference's ONNX-example layout) from PyTorch to
alexnet.onnx (reference: examples/python/onnx/alexnet_pt.py)."""
import torch
import torch.nn as nn
from _common import onnx_path

from flexflow.onnx.model import export_torch


class AlexNet(nn.Module):
    def __init__(self, num_classes=10):
        super().__init__()
        self.features = nn.Sequential(
            nn.Conv2d(3, 64, 11, 4, 2), nn.ReLU(inplace=True), nn.MaxPool2d(3, 2),
            nn.Conv2d(64, 192, 5, padding=2), nn.ReLU(inplace=True), nn.MaxPool2d(3, 2),
            nn.Conv2d(192, 384, 3, padding=1), nn.ReLU(inplace=True),
            nn.Conv2d(384, 256, 3, padding=1), nn.ReLU(inplace=True),
            nn.Conv2d(256, 256, 3, padding=1), nn.ReLU(inplace=True), nn.MaxPool2d(3, 2))
        self.classifier = nn.Sequential(
            nn.Linear(256 * 6 * 6, 4096), nn.ReLU(inplace=True), nn.Linear(4096, 4096), nn.ReLU(inplace=True),
            nn.Linear(4096, num_classes), nn.Softmax(dim=-1))

    def forward(self, x):
        return self.classifier(torch.flatten(self.features(x), 1))


def export(path=None):
    path = path or onnx_path("alexnet.onnx")
    export_torch(AlexNet(), torch.randn(2, 3, 224, 224), path, export_params=False)
    return path


if __name__ == "__main__":
    print("wrote", export())
