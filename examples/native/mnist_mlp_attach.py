"""MNIST MLP trained by an explicit loop that attaches every batch with
set_tensor (reference: examples/python/native/mnist_mlp_attach.py)."""
import numpy as np
from _common import num_samples, report

from flexflow.core import ActiMode, DataType, FFConfig, FFModel, LossType, MetricsType, SGDOptimizer
from flexflow.keras.datasets import mnist


def top_level_task():
    ffconfig = FFConfig()
    ffconfig.parse_args()
    m = FFModel(ffconfig)
    x = m.create_tensor([ffconfig.batch_size, 784], DataType.DT_FLOAT)
    t = m.dense(x, 512, ActiMode.AC_MODE_RELU)
    t = m.dense(t, 512, ActiMode.AC_MODE_RELU)
    t = m.softmax(m.dense(t, 10))
    m.optimizer = SGDOptimizer(m, 0.01)
    m.compile(loss_type=LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY,
              metrics=[MetricsType.METRICS_ACCURACY, MetricsType.METRICS_SPARSE_CATEGORICAL_CROSSENTROPY])
    n = num_samples(60000)
    (xt, yt), _ = mnist.load_data(num_samples=n)
    xt = xt.reshape(n, 784).astype("float32") / 255
    yt = np.reshape(yt.astype("int32"), (n, 1))
    label = m.label_tensor
    bs = ffconfig.batch_size
    m.init_layers()
    ts = ffconfig.get_current_time()
    for _ in range(ffconfig.epochs):
        m.reset_metrics()
        for it in range(n // bs):
            x.set_tensor(m, xt[it * bs:(it + 1) * bs])
            label.set_tensor(m, yt[it * bs:(it + 1) * bs])
            m.forward()
            m.zero_gradients()
            m.backward()
            m.update()
    report(ffconfig, ts, n, ffconfig.epochs)
    print(m.get_perf_metrics())
    print(m.get_layer_by_id(0).get_weight_tensor())


if __name__ == "__main__":
    print("mnist mlp attach")
    top_level_task()
