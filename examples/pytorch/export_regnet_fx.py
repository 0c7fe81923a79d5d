"""RegNetX in plain PyTorch (classy_vision is not installed here), followed
by Flatten + Linear as in the reference, exported to regnetX32gf.ff
(reference: examples/python/pytorch/export_regnet_fx.py).  Quick runs
(FF_EXAMPLE_SAMPLES set) export RegNetX-200MF instead of -32GF."""
import os

import torch.nn as nn
from _common import ff_path

from flexflow.torch.model import PyTorchModel

# (depths, widths, group width) of the RegNetX design space
CONFIGS = {"32gf": ([2, 7, 13, 1], [336, 672, 1344, 2520], 168), "200mf": ([1, 1, 4, 7], [24, 56, 152, 368], 8)}


class XBlock(nn.Module):
    def __init__(self, cin, cout, stride, group_width):
        super().__init__()
        groups = cout // group_width
        self.a = nn.Sequential(nn.Conv2d(cin, cout, 1, bias=False), nn.BatchNorm2d(cout), nn.ReLU(inplace=True))
        self.b = nn.Sequential(nn.Conv2d(cout, cout, 3, stride, 1, groups=groups, bias=False), nn.BatchNorm2d(cout),
                               nn.ReLU(inplace=True))
        self.c = nn.Sequential(nn.Conv2d(cout, cout, 1, bias=False), nn.BatchNorm2d(cout))
        self.proj = None
        if stride != 1 or cin != cout:
            self.proj = nn.Sequential(nn.Conv2d(cin, cout, 1, stride, bias=False), nn.BatchNorm2d(cout))
        self.relu = nn.ReLU(inplace=True)

    def forward(self, x):
        skip = self.proj(x) if self.proj is not None else x
        return self.relu(self.c(self.b(self.a(x))) + skip)


class RegNetX(nn.Module):
    def __init__(self, depths, widths, group_width):
        super().__init__()
        self.stem = nn.Sequential(nn.Conv2d(3, 32, 3, 2, 1, bias=False), nn.BatchNorm2d(32), nn.ReLU(inplace=True))
        blocks, cin = [], 32
        for d, w in zip(depths, widths):
            for i in range(d):
                blocks.append(XBlock(cin, w, 2 if i == 0 else 1, group_width))
                cin = w
        self.trunk = nn.Sequential(*blocks)
        self.out_channels = cin

    def forward(self, x):
        return self.trunk(self.stem(x))


def build(kind=None, image=224):
    kind = kind or ("200mf" if "FF_EXAMPLE_SAMPLES" in os.environ else "32gf")
    body = RegNetX(*CONFIGS[kind])
    side = image // 32
    return nn.Sequential(body, nn.Flatten(), nn.Linear(body.out_channels * side * side, 1000))


def export(path=None):
    path = path or ff_path("regnetX32gf.ff")
    PyTorchModel(build()).torch_to_file(path)
    return path


if __name__ == "__main__":
    print("wrote", export())
