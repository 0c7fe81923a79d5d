"""Recommendation / tabular benchmark models (FFModel API).

* DLRM — examples/cpp/DLRM/dlrm.cc:26-42,84-97,150-166: bottom MLP on dense
  features, one SUM-bag embedding per sparse feature (bag size 1), "cat"
  interaction, top MLP with a sigmoid on the last layer, MSE loss.  The
  run scripts' large config (8 tables x 1M rows, bot 64-512-512-64, top
  576-1024-1024-1024-1) is ``dlrm_large()``.  Tables can be placed on
  individual GPUs / sharded by the strategy search (parameter parallelism,
  §2.7) — the executor moves activations between the table-owning device
  set and the data-parallel MLPs.
* XDL — examples/cpp/XDL/xdl.cc: embeddings -> concat -> MLP 256-256-256-2.
* CANDLE-Uno — examples/cpp/candle_uno (feature towers 8 x 4192 on the
  cell/drug features, concat, 4 x 4192 dense, Dense(1), MSE).
* MLP_Unify — examples/cpp/MLP_Unify/mlp.cc:33-69 (two 8 x Dense(8192)
  towers on 1024-wide inputs, add, softmax).
"""
from __future__ import annotations

import dataclasses
import math
from typing import Dict, List, Tuple

import numpy as np

from ..core import ActiMode, AggrMode, DataType, FFModel
from ..core.initializers import NormInitializer, UniformInitializer, GlorotNormalInitializer


@dataclasses.dataclass
class DLRMConfig:
    batch_size: int = 256
    sparse_feature_size: int = 64
    embedding_size: List[int] = dataclasses.field(default_factory=lambda: [1000000] * 4)
    embedding_bag_size: int = 1
    mlp_bot: List[int] = dataclasses.field(default_factory=lambda: [4, 64, 64])
    mlp_top: List[int] = dataclasses.field(default_factory=lambda: [64, 64, 2])
    sigmoid_bot: int = -1
    sigmoid_top: int = -2  # index counted from the end: last layer
    arch_interaction_op: str = "cat"
    loss_threshold: float = 0.0
    dataset_path: str = ""
    data_size: int = -1

    @classmethod
    def from_args(cls, argv=None, **kw) -> "DLRMConfig":
        """The reference's DLRM command line (examples/cpp/DLRM/dlrm.cc
        parse_input_args): --arch-sparse-feature-size N, --arch-embedding-size
        a-b-c, --embedding-bag-size N, --arch-mlp-bot a-b-c, --arch-mlp-top
        a-b-c, --loss-threshold F, --sigmoid-top N, --sigmoid-bot N,
        --arch-interaction-op cat|dot, --dataset PATH, --data-size N, -b N."""
        import sys
        argv = sys.argv[1:] if argv is None else list(argv)
        cfg = cls(**kw)
        ints = lambda v: [int(x) for x in v.split("-") if x]  # noqa: E731
        flags = {"--arch-sparse-feature-size": ("sparse_feature_size", int),
                 "--arch-embedding-size": ("embedding_size", ints), "--embedding-bag-size": ("embedding_bag_size", int),
                 "--arch-mlp-bot": ("mlp_bot", ints), "--arch-mlp-top": ("mlp_top", ints),
                 "--loss-threshold": ("loss_threshold", float), "--sigmoid-top": ("sigmoid_top", int),
                 "--sigmoid-bot": ("sigmoid_bot", int), "--arch-interaction-op": ("arch_interaction_op", str),
                 "--dataset": ("dataset_path", str), "--data-size": ("data_size", int),
                 "-b": ("batch_size", int), "--batch-size": ("batch_size", int)}
        i = 0
        while i < len(argv):
            if argv[i] in flags and i + 1 < len(argv):
                name, conv = flags[argv[i]]
                setattr(cfg, name, conv(argv[i + 1]))
                i += 2
            else:
                i += 1
        return cfg


def dlrm_large(**kw) -> DLRMConfig:
    base = dict(embedding_size=[1000000] * 8, mlp_bot=[64, 512, 512, 64], mlp_top=[576, 1024, 1024, 1024, 1])
    base.update(kw)
    return DLRMConfig(**base)


def _mlp(model: FFModel, t, ln: List[int], sigmoid_layer: int, prefix: str):
    for i in range(len(ln) - 1):
        std = math.sqrt(2.0 / (ln[i + 1] + ln[i]))
        act = ActiMode.AC_MODE_SIGMOID if i == sigmoid_layer else ActiMode.AC_MODE_RELU
        t = model.dense(t, ln[i + 1], act, use_bias=False, kernel_initializer=NormInitializer(i, 0.0, std),
                        name=f"{prefix}{i}")
    return t


def build_dlrm(model: FFModel, cfg: DLRMConfig) -> Tuple[Dict[str, object], object]:
    B = cfg.batch_size
    sparse = [model.create_tensor([B, cfg.embedding_bag_size], DataType.DT_INT32, create_grad=False,
                                  name=f"sparse{i}") for i in range(len(cfg.embedding_size))]
    dense = model.create_tensor([B, cfg.mlp_bot[0]], DataType.DT_FLOAT, name="dense")
    x = _mlp(model, dense, cfg.mlp_bot, cfg.sigmoid_bot, "bot")
    ly = []
    for i, rows in enumerate(cfg.embedding_size):
        r = math.sqrt(1.0 / rows)
        ly.append(model.embedding(sparse[i], rows, cfg.sparse_feature_size, AggrMode.AGGR_MODE_SUM,
                                  kernel_initializer=UniformInitializer(i, -r, r), name=f"emb{i}"))
    z = model.concat([x] + ly, -1, name="interact")
    top = list(cfg.mlp_top)
    top[0] = model.cg.shape(z.vref).dims[-1]
    sig = cfg.sigmoid_top if cfg.sigmoid_top >= 0 else len(top) - 1 + cfg.sigmoid_top + 1
    p = _mlp(model, z, top, sig, "top")
    inputs = {f"sparse{i}": s for i, s in enumerate(sparse)}
    inputs["dense"] = dense
    return inputs, p


def dlrm_synthetic(cfg: DLRMConfig, rng: np.random.Generator):
    feeds = {f"sparse{i}": rng.integers(0, n, (cfg.batch_size, cfg.embedding_bag_size), dtype=np.int32)
             for i, n in enumerate(cfg.embedding_size)}
    feeds["dense"] = rng.random((cfg.batch_size, cfg.mlp_bot[0]), dtype=np.float32)
    y = rng.integers(0, 2, (cfg.batch_size, cfg.mlp_top[-1])).astype(np.float32)
    return feeds, y


@dataclasses.dataclass
class XDLConfig:
    batch_size: int = 256
    sparse_feature_size: int = 64
    embedding_size: List[int] = dataclasses.field(default_factory=lambda: [1000000] * 4)
    embedding_bag_size: int = 1
    mlp_top: List[int] = dataclasses.field(default_factory=lambda: [256, 256, 256, 2])


def build_xdl(model: FFModel, cfg: XDLConfig):
    B = cfg.batch_size
    sparse = [model.create_tensor([B, cfg.embedding_bag_size], DataType.DT_INT32, create_grad=False,
                                  name=f"sparse{i}") for i in range(len(cfg.embedding_size))]
    ly = []
    for i, rows in enumerate(cfg.embedding_size):
        r = math.sqrt(1.0 / rows)
        ly.append(model.embedding(sparse[i], rows, cfg.sparse_feature_size, AggrMode.AGGR_MODE_SUM,
                                  kernel_initializer=UniformInitializer(i, -r, r), name=f"emb{i}"))
    z = model.concat(ly, -1, name="interact")
    top = list(cfg.mlp_top)
    top[0] = model.cg.shape(z.vref).dims[-1]
    p = _mlp(model, z, top, len(top) - 2, "top")
    return {f"sparse{i}": s for i, s in enumerate(sparse)}, p


def xdl_synthetic(cfg: XDLConfig, rng: np.random.Generator):
    feeds = {f"sparse{i}": rng.integers(0, n, (cfg.batch_size, cfg.embedding_bag_size), dtype=np.int32)
             for i, n in enumerate(cfg.embedding_size)}
    return feeds, rng.integers(0, 2, (cfg.batch_size, cfg.mlp_top[-1])).astype(np.float32)


@dataclasses.dataclass
class CandleUnoConfig:
    batch_size: int = 64
    dense_layers: List[int] = dataclasses.field(default_factory=lambda: [4192] * 4)
    dense_feature_layers: List[int] = dataclasses.field(default_factory=lambda: [4192] * 8)
    feature_shapes: Dict[str, int] = dataclasses.field(default_factory=lambda: {
        "dose": 1, "cell.rnaseq": 942, "drug.descriptors": 5270, "drug.fingerprints": 2048})
    input_features: Dict[str, str] = dataclasses.field(default_factory=lambda: {
        "dose1": "dose", "dose2": "dose", "cell.rnaseq": "cell.rnaseq", "drug1.descriptors": "drug.descriptors",
        "drug1.fingerprints": "drug.fingerprints", "drug2.descriptors": "drug.descriptors",
        "drug2.fingerprints": "drug.fingerprints"})
    dropout: float = 0.1
    residual: bool = False


def build_candle_uno(model: FFModel, cfg: CandleUnoConfig):
    towers = {k for k in cfg.feature_shapes if "." in k and k.split(".")[0] in ("cell", "drug")}
    init = GlorotNormalInitializer(0)
    inputs, encoded = {}, []
    for name in sorted(cfg.input_features):
        feat = cfg.input_features[name]
        x = model.create_tensor([cfg.batch_size, cfg.feature_shapes[feat]], DataType.DT_FLOAT, name=name)
        inputs[name] = x
        t = x
        if feat in towers:
            for i, d in enumerate(cfg.dense_feature_layers):
                t = model.dense(t, d, ActiMode.AC_MODE_RELU, False, kernel_initializer=init, name=f"{name}.tower{i}")
                if cfg.dropout > 0:
                    t = model.dropout(t, cfg.dropout, i, name=f"{name}.tower{i}_dropout")
        encoded.append(t)
    out = model.concat(encoded, 1, name="concat")
    for i, d in enumerate(cfg.dense_layers):
        res = out
        out = model.dense(out, d, ActiMode.AC_MODE_RELU, False, kernel_initializer=init, name=f"dense{i}")
        if cfg.dropout > 0:
            out = model.dropout(out, cfg.dropout, 100 + i, name=f"dense{i}_dropout")
        if cfg.residual and res.dims == out.dims:
            out = model.add(out, res, name=f"dense{i}_residual")
    return inputs, model.dense(out, 1, ActiMode.AC_MODE_NONE, False, kernel_initializer=init, name="out")


def candle_uno_synthetic(cfg: CandleUnoConfig, rng: np.random.Generator):
    feeds = {n: rng.random((cfg.batch_size, cfg.feature_shapes[f]), dtype=np.float32)
             for n, f in cfg.input_features.items()}
    return feeds, rng.random((cfg.batch_size, 1), dtype=np.float32)


@dataclasses.dataclass
class MLPUnifyConfig:
    batch_size: int = 64
    input_dim: int = 1024
    hidden_dims: List[int] = dataclasses.field(default_factory=lambda: [8192] * 8)


def build_mlp_unify(model: FFModel, cfg: MLPUnifyConfig):
    x1 = model.create_tensor([cfg.batch_size, cfg.input_dim], DataType.DT_FLOAT, name="input1")
    x2 = model.create_tensor([cfg.batch_size, cfg.input_dim], DataType.DT_FLOAT, name="input2")
    t1, t2 = x1, x2
    n = len(cfg.hidden_dims)
    for i, d in enumerate(cfg.hidden_dims):
        act = ActiMode.AC_MODE_NONE if i == n - 1 else ActiMode.AC_MODE_RELU
        t1 = model.dense(t1, d, act, False, name=f"a{i}")
        t2 = model.dense(t2, d, act, False, name=f"b{i}")
    t = model.add(t1, t2, name="add")
    return {"input1": x1, "input2": x2}, model.softmax(t, name="softmax")


def mlp_unify_synthetic(cfg: MLPUnifyConfig, rng: np.random.Generator):
    feeds = {k: rng.standard_normal((cfg.batch_size, cfg.input_dim), dtype=np.float32) for k in ("input1", "input2")}
    return feeds, rng.integers(0, cfg.hidden_dims[-1], (cfg.batch_size, 1), dtype=np.int32)


def build_split_test(model: FFModel, batch_size: int = 64):
    """lib/models/src/models/split_test/split_test.cc:6-37."""
    x = model.create_tensor([batch_size, 256], DataType.DT_FLOAT, name="input")
    t = model.relu(model.dense(x, 128, name="fc0"), name="relu0")
    t = model.relu(model.add(model.dense(t, 64, name="fc1a"), model.dense(t, 64, name="fc1b"), name="add1"),
                   name="relu1")
    t = model.relu(model.add(model.dense(t, 32, name="fc2a"), model.dense(t, 32, name="fc2b"), name="add2"),
                   name="relu2")
    return {"input": x}, model.softmax(t, name="softmax")
