"""Plain-PyTorch ResNet-152 training loop, the eager baseline the reference
compares against (reference: examples/python/pytorch/resnet152_training.py;
synthetic CIFAR-shaped data at 224x224 instead of a torchvision download)."""
import os
import time

import torch
import torch.nn as nn
import torch.optim as optim
from _common import num_samples
from resnet_torch import resnet152, resnet18


def main():
    quick = "FF_EXAMPLE_SAMPLES" in os.environ
    device = "cuda:0" if torch.cuda.is_available() else "cpu"
    batch_size = 2 if quick else 4
    model = (resnet18 if quick else resnet152)(num_classes=10).to(device)
    criterion = nn.CrossEntropyLoss()
    optimizer = optim.SGD(model.parameters(), lr=0.001, momentum=0.9)
    g = torch.Generator().manual_seed(0)
    n = num_samples(10000)
    steps = max(1, n // batch_size)
    t0 = time.time()
    for i in range(steps):
        start = time.time()
        inputs = torch.rand(batch_size, 3, 224, 224, generator=g).to(device)
        labels = torch.randint(0, 10, (batch_size,), generator=g).to(device)
        optimizer.zero_grad()
        loss = criterion(model(inputs), labels)
        loss.backward()
        optimizer.step()
        print("Batch: %d Loss: %.3f Time per Image: %.5f" % (i, loss.item(), (time.time() - start) / batch_size))
    el = time.time() - t0
    print("ELAPSED TIME = %.4fs, THROUGHPUT = %.2f samples/s" % (el, steps * batch_size / el))


if __name__ == "__main__":
    main()
