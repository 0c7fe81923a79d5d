"""Convolutional benchmark models (FFModel API).

Parity with the reference's examples:
* AlexNet — examples/cpp/AlexNet/alexnet.cc:60-90 (3x229x229 input).
* ResNet-50 — examples/cpp/ResNet/resnet.cc:39-113 (bottleneck stages
  3-4-6-3, 229x229 input, the reference leaves BatchNorm commented out;
  ``batch_norm=True`` gives the standard network).
* ResNeXt-50 (32x4d) — examples/cpp/resnext50/resnext.cc (grouped 3x3).
* InceptionV3 — examples/cpp/InceptionV3/inception.cc and
  lib/models/src/models/inception_v3 (299x299; A x3, B, C x4, D, E x2).
"""
from __future__ import annotations

import dataclasses
from typing import Dict, Tuple

import numpy as np

from ..core import ActiMode, DataType, FFModel, PoolType


@dataclasses.dataclass
class CNNConfig:
    batch_size: int = 64
    image_size: int = 229
    num_classes: int = 10
    batch_norm: bool = True


def _image_input(model: FFModel, cfg: CNNConfig, size: int):
    return model.create_tensor([cfg.batch_size, 3, size, size], DataType.DT_FLOAT, name="image")


def build_alexnet(model: FFModel, cfg: CNNConfig) -> Tuple[Dict[str, object], object]:
    x = _image_input(model, cfg, cfg.image_size)
    R = ActiMode.AC_MODE_RELU
    t = model.conv2d(x, 64, 11, 11, 4, 4, 2, 2, R, name="conv1")
    t = model.pool2d(t, 3, 3, 2, 2, 0, 0, name="pool1")
    t = model.conv2d(t, 192, 5, 5, 1, 1, 2, 2, R, name="conv2")
    t = model.pool2d(t, 3, 3, 2, 2, 0, 0, name="pool2")
    t = model.conv2d(t, 384, 3, 3, 1, 1, 1, 1, R, name="conv3")
    t = model.conv2d(t, 256, 3, 3, 1, 1, 1, 1, R, name="conv4")
    t = model.conv2d(t, 256, 3, 3, 1, 1, 1, 1, R, name="conv5")
    t = model.pool2d(t, 3, 3, 2, 2, 0, 0, name="pool5")
    t = model.flat(t, name="flat")
    t = model.dense(t, 4096, R, name="fc6")
    t = model.dense(t, 4096, R, name="fc7")
    t = model.dense(t, cfg.num_classes, name="fc8")
    return {"image": x}, model.softmax(t, name="softmax")


class _Net:
    def __init__(self, model: FFModel, bn: bool):
        self.m, self.bn, self.n = model, bn, 0

    def conv(self, x, oc, k, s=1, p=0, relu=True, groups=1, kw=None, ph=None, pw=None):
        self.n += 1
        kh, kw = (k, k) if kw is None else (k, kw)
        ph = p if ph is None else ph
        pw = p if pw is None else pw
        if self.bn:
            t = self.m.conv2d(x, oc, kh, kw, s, s, ph, pw, ActiMode.AC_MODE_NONE, groups, False, name=f"conv{self.n}")
            return self.m.batch_norm(t, relu, name=f"bn{self.n}")
        act = ActiMode.AC_MODE_RELU if relu else ActiMode.AC_MODE_NONE
        return self.m.conv2d(x, oc, kh, kw, s, s, ph, pw, act, groups, True, name=f"conv{self.n}")


def _bottleneck(net: _Net, x, width, out_ch, stride, groups=1):
    t = net.conv(x, width, 1)
    t = net.conv(t, width, 3, stride, 1, groups=groups)
    t = net.conv(t, out_ch, 1, relu=False)
    in_ch = net.m.cg.shape(x.vref).dims[1]
    if stride != 1 or in_ch != out_ch:
        x = net.conv(x, out_ch, 1, stride, relu=False)
    net.n += 1
    return net.m.relu(net.m.add(x, t, name=f"res{net.n}"), False, name=f"relu{net.n}")


def _resnet(model: FFModel, cfg: CNNConfig, groups: int, width_per_group: int):
    net = _Net(model, cfg.batch_norm)
    x = _image_input(model, cfg, cfg.image_size)
    t = net.conv(x, 64, 7, 2, 3)
    t = model.pool2d(t, 3, 3, 2, 2, 1, 1, name="pool1")
    for stage, (blocks, planes) in enumerate(zip((3, 4, 6, 3), (64, 128, 256, 512))):
        width = planes if groups == 1 else groups * width_per_group * (2 ** stage)
        for b in range(blocks):
            t = _bottleneck(net, t, width, planes * 4, 2 if (b == 0 and stage > 0) else 1, groups)
    hw = model.cg.shape(t.vref).dims[-1]
    t = model.pool2d(t, hw, hw, 1, 1, 0, 0, PoolType.POOL_AVG, name="avgpool")
    t = model.flat(t, name="flat")
    t = model.dense(t, cfg.num_classes, name="fc")
    return {"image": x}, model.softmax(t, name="softmax")


def build_resnet50(model: FFModel, cfg: CNNConfig):
    return _resnet(model, cfg, 1, 64)


def build_resnext50(model: FFModel, cfg: CNNConfig):
    return _resnet(model, cfg, 32, 4)


def build_inception_v3(model: FFModel, cfg: CNNConfig):
    net = _Net(model, cfg.batch_norm)
    m = model
    cat_n = [0]

    def cat(xs):
        cat_n[0] += 1
        return m.concat(xs, 1, name=f"mixed{cat_n[0]}")

    def avg(x):
        net.n += 1
        return m.pool2d(x, 3, 3, 1, 1, 1, 1, PoolType.POOL_AVG, name=f"pool{net.n}")

    def maxp(x):
        net.n += 1
        return m.pool2d(x, 3, 3, 2, 2, 0, 0, name=f"pool{net.n}")

    c = net.conv

    def block_a(x, pf):
        return cat([c(x, 64, 1), c(c(x, 48, 1), 64, 5, p=2), c(c(c(x, 64, 1), 96, 3, p=1), 96, 3, p=1),
                    c(avg(x), pf, 1)])

    def block_b(x):
        return cat([c(x, 384, 3, 2), c(c(c(x, 64, 1), 96, 3, p=1), 96, 3, 2), maxp(x)])

    def block_c(x, c7):
        b7 = c(c(c(x, c7, 1), c7, 1, kw=7, ph=0, pw=3), 192, 7, kw=1, ph=3, pw=0)
        bd = c(x, c7, 1)
        for (kh, kw_, ph, pw, oc) in ((7, 1, 3, 0, c7), (1, 7, 0, 3, c7), (7, 1, 3, 0, c7), (1, 7, 0, 3, 192)):
            bd = c(bd, oc, kh, kw=kw_, ph=ph, pw=pw)
        return cat([c(x, 192, 1), b7, bd, c(avg(x), 192, 1)])

    def block_d(x):
        b3 = c(c(x, 192, 1), 320, 3, 2)
        b7 = c(c(c(x, 192, 1), 192, 1, kw=7, ph=0, pw=3), 192, 7, kw=1, ph=3, pw=0)
        return cat([b3, c(b7, 192, 3, 2), maxp(x)])

    def block_e(x):
        b3 = c(x, 384, 1)
        b3 = cat([c(b3, 384, 1, kw=3, ph=0, pw=1), c(b3, 384, 3, kw=1, ph=1, pw=0)])
        bd = c(c(x, 448, 1), 384, 3, p=1)
        bd = cat([c(bd, 384, 1, kw=3, ph=0, pw=1), c(bd, 384, 3, kw=1, ph=1, pw=0)])
        return cat([c(x, 320, 1), b3, bd, c(avg(x), 192, 1)])

    x = _image_input(model, cfg, 299 if cfg.image_size == 229 else cfg.image_size)
    t = c(x, 32, 3, 2)
    t = c(t, 32, 3)
    t = c(t, 64, 3, p=1)
    t = maxp(t)
    t = c(t, 80, 1)
    t = c(t, 192, 3)
    t = maxp(t)
    for pf in (32, 64, 64):
        t = block_a(t, pf)
    t = block_b(t)
    for c7 in (128, 160, 160, 192):
        t = block_c(t, c7)
    t = block_d(t)
    t = block_e(t)
    t = block_e(t)
    hw = m.cg.shape(t.vref).dims[-1]
    t = m.pool2d(t, hw, hw, 1, 1, 0, 0, PoolType.POOL_AVG, name="avgpool")
    t = m.flat(t, name="flat")
    t = m.dense(t, cfg.num_classes, name="fc")
    return {"image": x}, m.softmax(t, name="softmax")


def image_synthetic(model_inputs: Dict[str, object], cfg: CNNConfig, rng: np.random.Generator):
    x = model_inputs["image"]
    shp = x.dims
    return ({"image": rng.standard_normal(shp, dtype=np.float32)},
            rng.integers(0, cfg.num_classes, (shp[0], 1), dtype=np.int32))
