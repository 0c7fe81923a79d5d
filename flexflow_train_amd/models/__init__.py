"""Model zoo (FFModel builders for the reference's benchmark programs).

``MODELS[name] = (config_class, build_fn, synthetic_fn, loss, metrics)``;
``build(name, model, **cfg)`` builds into an FFModel and returns
(inputs, output, config).
"""
from __future__ import annotations

from typing import Callable, Dict, Tuple

from . import bert, cnn, moe, recsys, transformer

LOSS_CE = "sparse_categorical_crossentropy"
LOSS_MSE = "mean_squared_error"


def _bert_synth(cfg, rng):
    import numpy as np

    B, S = cfg.batch_size, cfg.sequence_length
    feeds = {"input_ids": rng.integers(0, cfg.vocab_size, (B, S), dtype=np.int32),
             "position_ids": np.broadcast_to(np.arange(S, dtype=np.int32), (B, S)).copy(),
             "token_type_ids": rng.integers(0, cfg.type_vocab_size, (B, S), dtype=np.int32)}
    return feeds, rng.integers(0, cfg.vocab_size, (B, S)).astype(np.int64)


MODELS: Dict[str, Tuple] = {
    "bert": (bert.BertConfig, bert.build_bert, _bert_synth, LOSS_CE),
    "transformer": (transformer.TransformerConfig, transformer.build_transformer, transformer.transformer_synthetic,
                    LOSS_MSE),
    "gpt": (transformer.GPTConfig, transformer.build_gpt, transformer.gpt_synthetic, LOSS_CE),
    "alexnet": (cnn.CNNConfig, cnn.build_alexnet, None, LOSS_CE),
    "resnet50": (cnn.CNNConfig, cnn.build_resnet50, None, LOSS_CE),
    "resnext50": (cnn.CNNConfig, cnn.build_resnext50, None, LOSS_CE),
    "inception_v3": (cnn.CNNConfig, cnn.build_inception_v3, None, LOSS_CE),
    "dlrm": (recsys.DLRMConfig, recsys.build_dlrm, recsys.dlrm_synthetic, LOSS_MSE),
    "xdl": (recsys.XDLConfig, recsys.build_xdl, recsys.xdl_synthetic, LOSS_MSE),
    "candle_uno": (recsys.CandleUnoConfig, recsys.build_candle_uno, recsys.candle_uno_synthetic, LOSS_MSE),
    "mlp_unify": (recsys.MLPUnifyConfig, recsys.build_mlp_unify, recsys.mlp_unify_synthetic, LOSS_CE),
    "moe": (moe.MoEConfig, moe.build_moe, moe.moe_synthetic, LOSS_CE),
}


def build(name: str, model, **cfg_kw):
    cfg_cls, fn, _, _ = MODELS[name]
    cfg = cfg_cls(**cfg_kw)
    inputs, out = fn(model, cfg)
    return inputs, out, cfg


def synthetic(name: str, cfg, inputs, rng):
    _, _, synth, _ = MODELS[name]
    if synth is None:
        return cnn.image_synthetic(inputs, cfg, rng)
    return synth(cfg, rng)


def loss_of(name: str) -> str:
    return MODELS[name][3]
