"""MNIST MLP through the native FFModel API: dense 512-512-10, SGD, data
loaders, fit + eval (reference: examples/python/native/mnist_mlp.py).
BASELINE config 1 (CPU plumbing) when run without a GPU."""
import numpy as np
from _common import num_samples, report

from flexflow.core import (ActiMode, DataType, FFConfig, FFModel, LossType, MetricsType, SGDOptimizer,
                           UniformInitializer)
from flexflow.keras.datasets import mnist


def top_level_task():
    ffconfig = FFConfig()
    ffconfig.parse_args()
    ffmodel = FFModel(ffconfig)
    x = ffmodel.create_tensor([ffconfig.batch_size, 784], DataType.DT_FLOAT)
    t = ffmodel.dense(x, 512, ActiMode.AC_MODE_RELU, kernel_initializer=UniformInitializer(12, -0.05, 0.05))
    t = ffmodel.dense(t, 512, ActiMode.AC_MODE_RELU)
    t = ffmodel.softmax(ffmodel.dense(t, 10))
    ffmodel.optimizer = SGDOptimizer(ffmodel, 0.01)
    ffmodel.compile(loss_type=LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY,
                    metrics=[MetricsType.METRICS_ACCURACY, MetricsType.METRICS_SPARSE_CATEGORICAL_CROSSENTROPY])
    n = num_samples(60000)
    (x_train, y_train), _ = mnist.load_data(num_samples=n)
    x_train = x_train.reshape(len(x_train), 784).astype("float32") / 255
    y_train = y_train.astype("int32").reshape(-1, 1)
    dl_x = ffmodel.create_data_loader(x, x_train)
    dl_y = ffmodel.create_data_loader(ffmodel.label_tensor, y_train)
    ffmodel.init_layers()
    ts = ffconfig.get_current_time()
    ffmodel.fit(x=dl_x, y=dl_y, epochs=ffconfig.epochs)
    ffmodel.eval(x=dl_x, y=dl_y)
    report(ffconfig, ts, len(x_train), ffconfig.epochs)
    return ffmodel.get_perf_metrics()


if __name__ == "__main__":
    pm = top_level_task()
    print("accuracy %.2f%%" % pm.get_accuracy())
