"""Import mnist_mlp_pt.onnx (--test_type 1) or mnist_mlp_keras.onnx
(--test_type 0) and train it on MNIST (reference: examples/python/onnx/mnist_mlp.py)."""
import os

import numpy as np
from _common import num_samples, onnx_path, report, test_type

from flexflow.core import DataType, FFConfig, FFModel, LossType, MetricsType, SGDOptimizer
from flexflow.keras.datasets import mnist
from flexflow.onnx.model import ONNXModel, ONNXModelKeras


def top_level_task(kind):
    ffconfig = FFConfig()
    ffconfig.parse_args()
    m = FFModel(ffconfig)
    x = m.create_tensor([ffconfig.batch_size, 784], DataType.DT_FLOAT)
    if kind == 1:
        path = onnx_path("mnist_mlp_pt.onnx")
        if not os.path.exists(path):
            from mnist_mlp_pt import export
            export(path)
        ONNXModel(path).apply(m, {"input.1": x})
    else:
        path = onnx_path("mnist_mlp_keras.onnx")
        if not os.path.exists(path):
            from mnist_mlp_keras import export
            export(path)
        ONNXModelKeras(path, ffconfig, m).apply(m, {"input_1": x})
    m.optimizer = SGDOptimizer(m, 0.01)
    m.compile(loss_type=LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY,
              metrics=[MetricsType.METRICS_ACCURACY, MetricsType.METRICS_SPARSE_CATEGORICAL_CROSSENTROPY])
    n = num_samples(60000)
    (xt, yt), _ = mnist.load_data(num_samples=n)
    dl_x = m.create_data_loader(x, xt.reshape(n, 784).astype("float32") / 255)
    dl_y = m.create_data_loader(m.label_tensor, np.reshape(yt.astype("int32"), (n, 1)))
    m.init_layers()
    ts = ffconfig.get_current_time()
    m.fit(x=dl_x, y=dl_y, epochs=ffconfig.epochs)
    report(ffconfig, ts, n, ffconfig.epochs)


if __name__ == "__main__":
    print("mnist mlp onnx")
    top_level_task(test_type())
