"""MNIST CNN through the native API (reference: examples/python/native/mnist_cnn.py)."""
import numpy as np
from _common import num_samples, report

from flexflow.core import ActiMode, DataType, FFConfig, FFModel, LossType, MetricsType, PoolType, SGDOptimizer
from flexflow.keras.datasets import mnist


def top_level_task():
    ffconfig = FFConfig()
    ffconfig.parse_args()
    m = FFModel(ffconfig)
    x = m.create_tensor([ffconfig.batch_size, 1, 28, 28], DataType.DT_FLOAT)
    R = ActiMode.AC_MODE_RELU
    t = m.conv2d(x, 32, 3, 3, 1, 1, 1, 1, R, True)
    t = m.conv2d(t, 64, 3, 3, 1, 1, 1, 1, R, True)
    t = m.pool2d(t, 2, 2, 2, 2, 0, 0, PoolType.POOL_MAX)
    t = m.flat(t)
    t = m.dense(t, 128, R)
    t = m.softmax(m.dense(t, 10))
    m.optimizer = SGDOptimizer(m, 0.01)
    m.compile(loss_type=LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY,
              metrics=[MetricsType.METRICS_ACCURACY, MetricsType.METRICS_SPARSE_CATEGORICAL_CROSSENTROPY])
    (xt, yt), _ = mnist.load_data(num_samples=num_samples(60000))
    xt = xt.reshape(len(xt), 1, 28, 28).astype("float32") / 255
    yt = np.reshape(yt.astype("int32"), (len(yt), 1))
    dl_x = m.create_data_loader(x, xt)
    dl_y = m.create_data_loader(m.label_tensor, yt)
    m.init_layers()
    ts = ffconfig.get_current_time()
    m.fit(x=dl_x, y=dl_y, epochs=ffconfig.epochs)
    report(ffconfig, ts, len(xt), ffconfig.epochs)


if __name__ == "__main__":
    print("mnist cnn")
    top_level_task()
