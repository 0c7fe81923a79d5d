"""Every model-zoo entry builds, compiles and takes a training step on CPU
at a tiny size (reference: the examples are the test programs run by
tests/multi_gpu_tests.sh)."""
import numpy as np
import pytest
import torch

from flexflow_train_amd import models as Z
from flexflow_train_amd.core import FFConfig, FFModel, LossType, MetricsType, SGDOptimizer

TINY = {
    "bert": dict(vocab_size=64, hidden_size=32, num_heads=4, dim_feedforward=64, num_encoder_layers=1,
                 sequence_length=8, batch_size=2, max_position_embeddings=8),
    "transformer": dict(hidden_size=32, num_heads=4, num_layers=2, sequence_length=8, batch_size=2),
    "gpt": dict(vocab_size=50, hidden_size=32, num_layers=2, num_heads=4, sequence_length=8, batch_size=2),
    "alexnet": dict(batch_size=2, image_size=67),
    "resnet50": dict(batch_size=2, image_size=32),
    "resnext50": dict(batch_size=2, image_size=32),
    "inception_v3": dict(batch_size=2, image_size=75),
    "dlrm": dict(batch_size=8, embedding_size=[100] * 3, mlp_bot=[4, 16, 16], mlp_top=[0, 16, 1]),
    "xdl": dict(batch_size=8, embedding_size=[100] * 3, sparse_feature_size=8, mlp_top=[0, 16, 16, 2]),
    "candle_uno": dict(batch_size=4, dense_layers=[32, 32], dense_feature_layers=[32, 32], dropout=0.0),
    "mlp_unify": dict(batch_size=4, input_dim=16, hidden_dims=[32, 32]),
    "moe": dict(batch_size=4, input_dim=16, expert_hidden=16, num_experts=4, num_classes=5),
}


@pytest.mark.parametrize("name", sorted(TINY))
def test_model_trains_one_step(name):
    cfg = FFConfig()
    m = FFModel(cfg)
    inputs, out, mcfg = Z.build(name, m, **TINY[name])
    loss = Z.loss_of(name)
    lt = (LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY if loss == Z.LOSS_CE
          else LossType.LOSS_MEAN_SQUARED_ERROR_AVG_REDUCE)
    m.compile(optimizer=SGDOptimizer(m, lr=0.01), loss_type=lt, metrics=[MetricsType.METRICS_ACCURACY]
              if loss == Z.LOSS_CE else [MetricsType.METRICS_MEAN_SQUARED_ERROR])
    feeds, labels = Z.synthetic(name, mcfg, inputs, np.random.default_rng(0))
    ex = m.executor
    feeds = {k: torch.as_tensor(v) for k, v in feeds.items()}
    ex.train_step(feeds, torch.as_tensor(labels))
    ex.zero_metrics()
    ex.train_step(feeds, torch.as_tensor(labels))
    pm = ex.perf_metrics()
    assert np.isfinite(pm.loss) and pm.train_all > 0
