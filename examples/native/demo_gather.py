"""Gather of dense-layer rows by a neighbour index, trained with
forward / backward / update (reference: examples/python/native/demo_gather.py)."""
import numpy as np
from _common import report

from flexflow.core import ActiMode, DataType, FFConfig, FFModel, LossType, MetricsType, SGDOptimizer


def top_level_task():
    ffconfig = FFConfig()
    ffconfig.parse_args()
    bs = ffconfig.batch_size
    m = FFModel(ffconfig)
    neighbors = np.array([[[0], [5], [3], [3], [7], [9]]]).repeat(bs, 0).repeat(5, 2).astype(np.int32)
    xv = np.full((bs, 16, 5), 0.01, np.float32)
    inp = m.create_tensor([bs, 16, 5], DataType.DT_FLOAT)
    index = m.create_tensor([bs, 6, 5], DataType.DT_INT32)
    x0 = m.dense(inp, 5, ActiMode.AC_MODE_NONE, False)
    m.gather(x0, index, 1)
    m.optimizer = SGDOptimizer(m, 0.01)
    m.compile(loss_type=LossType.LOSS_MEAN_SQUARED_ERROR_AVG_REDUCE, metrics=[MetricsType.METRICS_MEAN_SQUARED_ERROR])
    m.init_layers()
    inp.attach_numpy_array(m, ffconfig, xv)
    index.attach_numpy_array(m, ffconfig, neighbors)
    m.label_tensor.attach_numpy_array(m, ffconfig, np.random.default_rng(0).random((bs, 6, 5)).astype("float32"))
    ts = ffconfig.get_current_time()
    steps = 100
    for _ in range(steps):
        m.forward()
        m.zero_gradients()
        m.backward()
        m.update()
    print(m.get_perf_metrics())
    report(ffconfig, ts, bs * steps, 1)


if __name__ == "__main__":
    print("Demo Gather")
    top_level_task()
