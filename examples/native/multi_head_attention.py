"""Multi-head self-attention block regressed onto a target with MSE
(reference: examples/python/native/multi_head_attention.py)."""
import numpy as np
from _common import num_samples, report

from flexflow.core import DataType, FFConfig, FFModel, LossType, MetricsType, SGDOptimizer


def top_level_task():
    ffconfig = FFConfig()
    ffconfig.parse_args()
    m = FFModel(ffconfig)
    seq, hidden, heads = 64, 256, 8
    q = m.create_tensor([ffconfig.batch_size, seq, hidden], DataType.DT_FLOAT)
    t = m.multihead_attention(q, q, q, hidden, heads, hidden // heads, hidden // heads)
    t = m.dense(t, hidden)
    m.optimizer = SGDOptimizer(m, 0.001)
    m.compile(loss_type=LossType.LOSS_MEAN_SQUARED_ERROR_AVG_REDUCE, metrics=[MetricsType.METRICS_MEAN_SQUARED_ERROR])
    n = num_samples(1024)
    rng = np.random.default_rng(0)
    xs = rng.standard_normal((n, seq, hidden)).astype("float32")
    ys = rng.standard_normal((n, seq, hidden)).astype("float32") * 0.1
    ts = ffconfig.get_current_time()
    m.fit(x=xs, y=ys, epochs=ffconfig.epochs)
    report(ffconfig, ts, n, ffconfig.epochs)


if __name__ == "__main__":
    top_level_task()
