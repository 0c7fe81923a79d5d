"""Export a two-input CIFAR-10 CNN (shared first conv, concat / split) to
the .ff text IR (reference: examples/python/pytorch/cifar10_cnn_torch.py;
the split here is along channels, which is what the concat produced)."""
import torch
import torch.nn as nn
from _common import ff_path

from flexflow.torch.model import PyTorchModel


class CNN(nn.Module):
    def __init__(self):
        super().__init__()
        self.conv1 = nn.Conv2d(3, 32, 3, 1)
        self.conv2 = nn.Conv2d(64, 32, 3, 1)
        self.pool1 = nn.MaxPool2d(2, 2)
        self.conv3 = nn.Conv2d(32, 64, 3, 1)
        self.conv4 = nn.Conv2d(64, 64, 3, 1)
        self.pool2 = nn.MaxPool2d(2, 2)
        self.flat1 = nn.Flatten()
        self.linear1 = nn.Linear(1600, 512)
        self.linear2 = nn.Linear(512, 10)
        self.relu = nn.ReLU()

    def forward(self, input1, input2):
        y1 = self.relu(self.conv1(input1))
        y2 = self.relu(self.conv1(input2))
        y = torch.cat((y1, y2), 1)
        (y1, y2) = torch.split(y, 32, 1)
        y = torch.cat((y1, y2), 1)
        y = self.pool1(self.relu(self.conv2(y)))
        y = self.relu(self.conv3(y))
        y = self.pool2(self.relu(self.conv4(y)))
        y = self.relu(self.linear1(self.flat1(y)))
        return self.linear2(y), y


def export(path=None):
    path = path or ff_path("cnn.ff")
    PyTorchModel(CNN()).torch_to_file(path)
    return path


if __name__ == "__main__":
    print("wrote", export())
