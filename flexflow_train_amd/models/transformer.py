"""Transformer-family training models built through the FFModel API.

* ``build_transformer`` — the reference's AE "Transformer" benchmark
  (examples/cpp/Transformer/transformer.cc:33-45,78-84,159-211): N encoder
  blocks of self-attention followed by two bias-free dense layers (ReLU,
  then linear), a final Dense(1), MSE loss, SGD lr 0.01; hidden 1024,
  16 heads, 12 layers, seq 512 by default.
* ``build_gpt`` — decoder-only causal LM (GPT-2/3 layout: pre-LayerNorm
  blocks, GELU MLP 4x, learned positions, causal flash attention).
  ``gpt3_medium()`` = 24 layers x 1024, 16 heads, seq 2048, vocab 50257.
"""
from __future__ import annotations

import dataclasses
from typing import Dict, Tuple

import numpy as np

from ..core import ActiMode, AggrMode, DataType, FFModel
from ..core.initializers import NormInitializer, ZeroInitializer


@dataclasses.dataclass
class TransformerConfig:
    hidden_size: int = 1024
    num_heads: int = 16
    num_layers: int = 12
    sequence_length: int = 512
    batch_size: int = 64


def build_transformer(model: FFModel, cfg: TransformerConfig) -> Tuple[Dict[str, object], object]:
    B, S, H = cfg.batch_size, cfg.sequence_length, cfg.hidden_size
    x = model.create_tensor([B, S, H], DataType.DT_FLOAT, name="input")
    t = x
    d = H // cfg.num_heads
    for i in range(cfg.num_layers):
        t = model.multihead_attention(t, t, t, H, cfg.num_heads, d, d, name=f"layer{i}.attn")
        t = model.dense(t, H, ActiMode.AC_MODE_RELU, use_bias=False, name=f"layer{i}.fc1")
        t = model.dense(t, H, ActiMode.AC_MODE_NONE, use_bias=False, name=f"layer{i}.fc2")
    out = model.dense(t, 1, ActiMode.AC_MODE_NONE, use_bias=False, name="out")
    return {"input": x}, out


def transformer_synthetic(cfg: TransformerConfig, rng: np.random.Generator):
    x = rng.standard_normal((cfg.batch_size, cfg.sequence_length, cfg.hidden_size), dtype=np.float32)
    y = rng.standard_normal((cfg.batch_size, cfg.sequence_length, 1), dtype=np.float32)
    return {"input": x}, y


@dataclasses.dataclass
class GPTConfig:
    vocab_size: int = 50257
    hidden_size: int = 1024
    num_layers: int = 24
    num_heads: int = 16
    sequence_length: int = 2048
    batch_size: int = 8
    ffn_mult: int = 4
    layer_norm_eps: float = 1e-5
    initializer_range: float = 0.02
    pad_vocab_to: int = 64

    @property
    def padded_vocab(self) -> int:
        p = self.pad_vocab_to
        return (self.vocab_size + p - 1) // p * p


def gpt3_medium(**kw) -> GPTConfig:
    return GPTConfig(**kw)


def build_gpt(model: FFModel, cfg: GPTConfig) -> Tuple[Dict[str, object], object]:
    B, S, E = cfg.batch_size, cfg.sequence_length, cfg.hidden_size
    init = NormInitializer(0, 0.0, cfg.initializer_range)
    zero = ZeroInitializer()
    tok = model.create_tensor([B, S], DataType.DT_INT32, create_grad=False, name="input_ids")
    pos = model.create_tensor([B, S], DataType.DT_INT32, create_grad=False, name="position_ids")
    x = model.add(model.embedding(tok, cfg.padded_vocab, E, AggrMode.AGGR_MODE_NONE, kernel_initializer=init,
                                  name="wte"),
                  model.embedding(pos, S, E, AggrMode.AGGR_MODE_NONE, kernel_initializer=init, name="wpe"),
                  name="embed_add")
    for i in range(cfg.num_layers):
        p = f"h{i}"
        h = model.layer_norm(x, [-1], True, cfg.layer_norm_eps, name=f"{p}.ln1")
        a = model.multihead_attention(h, h, h, E, cfg.num_heads, bias=True, kernel_initializer=init, causal=True,
                                      name=f"{p}.attn")
        x = model.add(x, a, name=f"{p}.attn_residual")
        h = model.layer_norm(x, [-1], True, cfg.layer_norm_eps, name=f"{p}.ln2")
        h = model.dense(h, cfg.ffn_mult * E, ActiMode.AC_MODE_GELU, True, kernel_initializer=init,
                        bias_initializer=zero, name=f"{p}.fc")
        h = model.dense(h, E, ActiMode.AC_MODE_NONE, True, kernel_initializer=init, bias_initializer=zero,
                        name=f"{p}.proj")
        x = model.add(x, h, name=f"{p}.mlp_residual")
    x = model.layer_norm(x, [-1], True, cfg.layer_norm_eps, name="ln_f")
    logits = model.dense(x, cfg.padded_vocab, ActiMode.AC_MODE_NONE, False, kernel_initializer=init,
                         name="lm_head")
    probs = model.softmax(logits, -1, name="softmax")
    model.valid_classes = cfg.vocab_size
    return {"input_ids": tok, "position_ids": pos}, probs


def gpt_synthetic(cfg: GPTConfig, rng: np.random.Generator):
    B, S = cfg.batch_size, cfg.sequence_length
    ids = rng.integers(0, cfg.vocab_size, (B, S + 1), dtype=np.int32)
    pos = np.broadcast_to(np.arange(S, dtype=np.int32), (B, S)).copy()
    return {"input_ids": ids[:, :S].copy(), "position_ids": pos}, ids[:, 1:].astype(np.int64)
