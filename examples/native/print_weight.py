"""Read a dense layer's weights after init (a uniform(-1, 1) kernel
initializer) (reference: examples/python/native/print_weight.py)."""
import numpy as np
from _common import num_samples

from flexflow.core import (ActiMode, DataType, FFConfig, FFModel, LossType, MetricsType, SGDOptimizer,
                           UniformInitializer)
from flexflow.keras.datasets import mnist


def top_level_task():
    ffconfig = FFConfig()
    ffconfig.parse_args()
    m = FFModel(ffconfig)
    x = m.create_tensor([ffconfig.batch_size, 784], DataType.DT_FLOAT)
    t = m.dense(x, 512, ActiMode.AC_MODE_RELU, kernel_initializer=UniformInitializer(12, -1, 1))
    t = m.dense(t, 512, ActiMode.AC_MODE_RELU)
    m.softmax(m.dense(t, 10))
    m.optimizer = SGDOptimizer(m, 0.01)
    m.compile(loss_type=LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY,
              metrics=[MetricsType.METRICS_ACCURACY, MetricsType.METRICS_SPARSE_CATEGORICAL_CROSSENTROPY])
    n = num_samples(60000)
    (xt, yt), _ = mnist.load_data(num_samples=n)
    m.create_data_loader(x, xt.reshape(n, 784).astype("float32") / 255)
    m.create_data_loader(m.label_tensor, np.reshape(yt.astype("int32"), (n, 1)))
    m.init_layers()
    dense1 = m.get_layer_by_id(0)
    w = dense1.get_weight_tensor().get_weights(m)
    print(dense1, dense1.get_weight_tensor(), w.shape, float(w.min()), float(w.max()))
    assert -1.0 <= w.min() < -0.9 and 0.9 < w.max() <= 1.0
    print("THROUGHPUT = n/a (weight inspection only)")


if __name__ == "__main__":
    print("mnist mlp test weight")
    top_level_task()
