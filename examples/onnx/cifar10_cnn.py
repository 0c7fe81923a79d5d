"""Import cifar10_cnn_pt.onnx (--test_type 1) or cifar10_cnn_keras.onnx
(--test_type 0) and train on CIFAR-10 (reference: examples/python/onnx/cifar10_cnn.py)."""
import os

from _common import num_samples, onnx_path, report, test_type

from flexflow.core import DataType, FFConfig, FFModel, LossType, MetricsType, SGDOptimizer
from flexflow.keras.datasets import cifar10
from flexflow.onnx.model import ONNXModel, ONNXModelKeras


def top_level_task(kind):
    ffconfig = FFConfig()
    ffconfig.parse_args()
    m = FFModel(ffconfig)
    x = m.create_tensor([ffconfig.batch_size, 3, 32, 32], DataType.DT_FLOAT)
    name = "cifar10_cnn_pt.onnx" if kind == 1 else "cifar10_cnn_keras.onnx"
    path = onnx_path(name)
    if not os.path.exists(path):
        if kind == 1:
            from cifar10_cnn_pt import export
        else:
            from cifar10_cnn_keras import export
        export(path)
    if kind == 1:
        ONNXModel(path).apply(m, {"input.1": x})
    else:
        ONNXModelKeras(path, ffconfig, m).apply(m, {"input_1": x})
    m.optimizer = SGDOptimizer(m, 0.01)
    m.compile(loss_type=LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY,
              metrics=[MetricsType.METRICS_ACCURACY, MetricsType.METRICS_SPARSE_CATEGORICAL_CROSSENTROPY])
    (xt, yt), _ = cifar10.load_data(num_samples(10000))
    dl_x = m.create_data_loader(x, xt.astype("float32") / 255)
    dl_y = m.create_data_loader(m.label_tensor, yt.astype("int32"))
    m.init_layers()
    ts = ffconfig.get_current_time()
    m.fit(x=dl_x, y=dl_y, epochs=ffconfig.epochs)
    report(ffconfig, ts, dl_x.num_samples, ffconfig.epochs)


if __name__ == "__main__":
    print("cifar10 cnn onnx")
    top_level_task(test_type())
