"""DLRM: per-table embeddings + bottom MLP, concat interaction, top MLP with
sigmoid, MSE (reference: examples/python/native/dlrm.py, examples/cpp/DLRM).
On several GPUs compile() may place tables on different ranks (parameter
parallel) with all-to-all exchanges, as searched."""
import numpy as np
from _common import num_samples, report

from flexflow.core import FFConfig, FFModel, LossType, MetricsType, SGDOptimizer
from flexflow_train_amd.models.recsys import DLRMConfig, build_dlrm, dlrm_synthetic


def top_level_task():
    ffconfig = FFConfig()
    ffconfig.parse_args()
    cfg = DLRMConfig(batch_size=ffconfig.batch_size, embedding_size=[100000] * 4, mlp_bot=[16, 64, 64],
                     mlp_top=[320, 64, 1])
    m = FFModel(ffconfig)
    inputs, out = build_dlrm(m, cfg)
    m.optimizer = SGDOptimizer(m, 0.01)
    m.compile(loss_type=LossType.LOSS_MEAN_SQUARED_ERROR_AVG_REDUCE, metrics=[MetricsType.METRICS_MEAN_SQUARED_ERROR])
    n = num_samples(32 * ffconfig.batch_size)
    cfg_all = DLRMConfig(**{**cfg.__dict__, "batch_size": n})
    feeds, y = dlrm_synthetic(cfg_all, np.random.default_rng(0))
    xs = [feeds[t.name] for t in m._inputs]
    ts = ffconfig.get_current_time()
    m.fit(x=xs, y=y, epochs=ffconfig.epochs)
    report(ffconfig, ts, n, ffconfig.epochs)


if __name__ == "__main__":
    top_level_task()
