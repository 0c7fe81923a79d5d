"""BERT (encoder-only transformer) built on the FFModel API.

Parity: lib/models/src/models/bert/bert.cc:25-158 (post-LN encoder layers:
MHA -> add -> LayerNorm -> FFN(GELU) -> add -> LayerNorm; a dense + softmax
head over the vocabulary) and get_default_bert_config (:8-23).  Additions
for a trainable MLM benchmark: token / position / segment embeddings and the
standard BERT transform (dense + GELU + LayerNorm) before the vocabulary
projection.  The reference's kdim = dim_feedforward / num_heads quirk is not
reproduced (kdim = hidden / heads).

The vocabulary is padded to a multiple of 64 (30522 -> 30528) so logits rows
are 16-byte aligned for the vector loads of the fused softmax-CE kernel;
padded classes are masked out of the softmax (valid_classes).
"""
from __future__ import annotations

import dataclasses
from typing import Dict, Tuple

from ..core import ActiMode, AggrMode, DataType, FFModel
from ..core.initializers import NormInitializer, TruncatedNormalInitializer, ZeroInitializer


@dataclasses.dataclass
class BertConfig:
    vocab_size: int = 30522
    hidden_size: int = 768
    num_encoder_layers: int = 12
    num_heads: int = 12
    dim_feedforward: int = 3072
    hidden_act: str = "gelu"
    hidden_dropout_prob: float = 0.0
    attention_probs_dropout_prob: float = 0.0
    initializer_range: float = 0.02
    layer_norm_eps: float = 1e-12
    sequence_length: int = 512
    batch_size: int = 64
    type_vocab_size: int = 2
    max_position_embeddings: int = 512
    embeddings: bool = True          # False -> hidden-state input like the reference graph
    mlm_transform: bool = True
    pad_vocab_to: int = 64

    @property
    def padded_vocab(self) -> int:
        p = self.pad_vocab_to
        return (self.vocab_size + p - 1) // p * p


def bert_base(**kw) -> BertConfig:
    return BertConfig(**kw)


def bert_large(**kw) -> BertConfig:
    base = dict(hidden_size=1024, num_encoder_layers=24, num_heads=16, dim_feedforward=4096)
    base.update(kw)
    return BertConfig(**base)


def build_bert(model: FFModel, cfg: BertConfig) -> Tuple[Dict[str, object], object]:
    B, S, E = cfg.batch_size, cfg.sequence_length, cfg.hidden_size
    proj_init = TruncatedNormalInitializer(0, 0.0, cfg.initializer_range, -2 * cfg.initializer_range,
                                           2 * cfg.initializer_range)
    emb_init = NormInitializer(0, 0.0, cfg.initializer_range)
    zero = ZeroInitializer()
    inputs = {}
    if cfg.embeddings:
        tok = model.create_tensor([B, S], DataType.DT_INT32, create_grad=False, name="input_ids")
        pos = model.create_tensor([B, S], DataType.DT_INT32, create_grad=False, name="position_ids")
        typ = model.create_tensor([B, S], DataType.DT_INT32, create_grad=False, name="token_type_ids")
        inputs.update(input_ids=tok, position_ids=pos, token_type_ids=typ)
        e = model.embedding(tok, cfg.padded_vocab, E, AggrMode.AGGR_MODE_NONE, kernel_initializer=emb_init,
                            name="embeddings.word")
        p = model.embedding(pos, cfg.max_position_embeddings, E, AggrMode.AGGR_MODE_NONE,
                            kernel_initializer=emb_init, name="embeddings.position")
        t = model.embedding(typ, cfg.type_vocab_size, E, AggrMode.AGGR_MODE_NONE, kernel_initializer=emb_init,
                            name="embeddings.token_type")
        x = model.add(model.add(e, p, name="embeddings.add0"), t, name="embeddings.add1")
        x = model.layer_norm(x, [-1], True, cfg.layer_norm_eps, name="embeddings.ln")
    else:
        x = model.create_tensor([B, S, E], DataType.DT_FLOAT, create_grad=True, name="hidden_input")
        inputs["hidden_input"] = x
    act = ActiMode.AC_MODE_GELU if cfg.hidden_act == "gelu" else ActiMode.AC_MODE_RELU
    for i in range(cfg.num_encoder_layers):
        pre = f"encoder.{i}"
        a = model.multihead_attention(x, x, x, E, cfg.num_heads, dropout=cfg.attention_probs_dropout_prob,
                                      bias=True, kernel_initializer=proj_init, name=f"{pre}.attn")
        if cfg.hidden_dropout_prob > 0:
            a = model.dropout(a, cfg.hidden_dropout_prob, i, name=f"{pre}.attn_dropout")
        x = model.layer_norm(model.add(a, x, name=f"{pre}.attn_residual"), [-1], True, cfg.layer_norm_eps,
                             name=f"{pre}.attn_ln")
        f = model.dense(x, cfg.dim_feedforward, act, True, kernel_initializer=proj_init, bias_initializer=zero,
                        name=f"{pre}.ffn1")
        f = model.dense(f, E, ActiMode.AC_MODE_NONE, True, kernel_initializer=proj_init, bias_initializer=zero,
                        name=f"{pre}.ffn2")
        if cfg.hidden_dropout_prob > 0:
            f = model.dropout(f, cfg.hidden_dropout_prob, 1000 + i, name=f"{pre}.ffn_dropout")
        x = model.layer_norm(model.add(f, x, name=f"{pre}.ffn_residual"), [-1], True, cfg.layer_norm_eps,
                             name=f"{pre}.ffn_ln")
    if cfg.mlm_transform:
        x = model.dense(x, E, act, True, kernel_initializer=proj_init, bias_initializer=zero, name="mlm.transform")
        x = model.layer_norm(x, [-1], True, cfg.layer_norm_eps, name="mlm.ln")
    logits = model.dense(x, cfg.padded_vocab, ActiMode.AC_MODE_NONE, True, kernel_initializer=proj_init,
                         bias_initializer=zero, name="mlm.decoder")
    probs = model.softmax(logits, -1, name="mlm.softmax")
    model.valid_classes = cfg.vocab_size
    return inputs, probs
