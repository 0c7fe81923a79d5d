"""BERT-like encoder proxy: L x (MHA + residual LayerNorm + GELU FFN),
synthetic tokens (reference: examples/python/native/bert_proxy_native.py).
Flags: -b batch, -e epochs, --layers/--hidden/--seq via FF flags."""
import argparse

import numpy as np
from _common import num_samples, report

from flexflow.core import (ActiMode, AdamOptimizer, AggrMode, DataType, FFConfig, FFModel, LossType, MetricsType)


def top_level_task():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layers", type=int, default=2)
    ap.add_argument("--hidden", type=int, default=256)
    ap.add_argument("--heads", type=int, default=4)
    ap.add_argument("--seq", type=int, default=128)
    ap.add_argument("--vocab", type=int, default=1024)
    args, rest = ap.parse_known_args()
    ffconfig = FFConfig()
    ffconfig.parse_args(rest)
    m = FFModel(ffconfig)
    B, S, E = ffconfig.batch_size, args.seq, args.hidden
    tok = m.create_tensor([B, S], DataType.DT_INT32)
    x = m.embedding(tok, args.vocab, E, AggrMode.AGGR_MODE_NONE)
    for _ in range(args.layers):
        a = m.multihead_attention(x, x, x, E, args.heads, E // args.heads, E // args.heads)
        x = m.layer_norm(m.add(x, a), [-1])
        f = m.dense(m.dense(x, 4 * E, ActiMode.AC_MODE_GELU), E)
        x = m.layer_norm(m.add(x, f), [-1])
    m.softmax(m.dense(x, args.vocab))
    m.optimizer = AdamOptimizer(m, alpha=1e-4)
    m.compile(loss_type=LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY,
              metrics=[MetricsType.METRICS_ACCURACY, MetricsType.METRICS_SPARSE_CATEGORICAL_CROSSENTROPY])
    n = num_samples(16 * B)
    rng = np.random.default_rng(0)
    ids = rng.integers(0, args.vocab, (n, S)).astype("int32")
    ts = ffconfig.get_current_time()
    m.fit(x=ids, y=np.roll(ids, 1, axis=1).astype("int32"), epochs=ffconfig.epochs)
    report(ffconfig, ts, n, ffconfig.epochs)


if __name__ == "__main__":
    top_level_task()
