"""SqueezeNet 1.1 in plain PyTorch (torchvision's layout; torchvision is not
installed here) exported to squeezenet.ff (reference:
examples/python/pytorch/torch_vision_torch.py)."""
import torch
import torch.nn as nn
from _common import ff_path

from flexflow.torch.model import PyTorchModel


class Fire(nn.Module):
    def __init__(self, cin, squeeze, e1, e3):
        super().__init__()
        self.squeeze = nn.Conv2d(cin, squeeze, 1)
        self.expand1x1 = nn.Conv2d(squeeze, e1, 1)
        self.expand3x3 = nn.Conv2d(squeeze, e3, 3, padding=1)
        self.relu = nn.ReLU(inplace=True)

    def forward(self, x):
        x = self.relu(self.squeeze(x))
        return torch.cat([self.relu(self.expand1x1(x)), self.relu(self.expand3x3(x))], 1)


class SqueezeNet(nn.Module):
    def __init__(self, num_classes=10):
        super().__init__()
        self.features = nn.Sequential(
            nn.Conv2d(3, 64, 3, 2), nn.ReLU(inplace=True), nn.MaxPool2d(3, 2),
            Fire(64, 16, 64, 64), Fire(128, 16, 64, 64), nn.MaxPool2d(3, 2),
            Fire(128, 32, 128, 128), Fire(256, 32, 128, 128), nn.MaxPool2d(3, 2),
            Fire(256, 48, 192, 192), Fire(384, 48, 192, 192), Fire(384, 64, 256, 256), Fire(512, 64, 256, 256))
        self.classifier = nn.Sequential(nn.Dropout(0.5), nn.Conv2d(512, num_classes, 1), nn.ReLU(inplace=True),
                                        nn.AdaptiveAvgPool2d((1, 1)))
        self.flat = nn.Flatten()
        self.softmax = nn.Softmax(dim=-1)

    def forward(self, x):
        return self.softmax(self.flat(self.classifier(self.features(x))))


def export(path=None):
    path = path or ff_path("squeezenet.ff")
    PyTorchModel(SqueezeNet()).torch_to_file(path)
    return path


if __name__ == "__main__":
    print("wrote", export())
