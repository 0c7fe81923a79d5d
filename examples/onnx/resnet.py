"""Import resnet18.onnx and train it on CIFAR-10 upsampled to 229x229
(reference: examples/python/onnx/resnet.py)."""
import os

from _common import num_samples, onnx_path, report, upsample

from flexflow.core import DataType, FFConfig, FFModel, LossType, MetricsType, SGDOptimizer
from flexflow.keras.datasets import cifar10
from flexflow.onnx.model import ONNXModel


def top_level_task():
    path = onnx_path("resnet18.onnx")
    if not os.path.exists(path):
        from resnet_pt import export
        export(path)
    ffconfig = FFConfig()
    ffconfig.parse_args()
    m = FFModel(ffconfig)
    x = m.create_tensor([ffconfig.batch_size, 3, 229, 229], DataType.DT_FLOAT)
    t = ONNXModel(path).apply(m, {"input.1": x})
    m.softmax(t)
    m.optimizer = SGDOptimizer(m, 0.01)
    m.compile(loss_type=LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY,
              metrics=[MetricsType.METRICS_ACCURACY, MetricsType.METRICS_SPARSE_CATEGORICAL_CROSSENTROPY])
    (xt, yt), _ = cifar10.load_data(num_samples(10000))
    dl_x = m.create_data_loader(x, upsample(xt, 229).astype("float32") / 255)
    dl_y = m.create_data_loader(m.label_tensor, yt.astype("int32"))
    m.init_layers()
    ts = ffconfig.get_current_time()
    m.fit(x=dl_x, y=dl_y, epochs=ffconfig.epochs)
    report(ffconfig, ts, dl_x.num_samples, ffconfig.epochs)


if __name__ == "__main__":
    print("resnet onnx")
    top_level_task()
