"""Rebuild the exported two-input CNN from cnn.ff and train it on CIFAR-10
(reference: examples/python/pytorch/cifar10_cnn.py; run cifar10_cnn_torch.py
first, or let this script export it)."""
import os

from _common import ff_path, num_samples, report

from flexflow.core import DataType, FFConfig, FFModel, LossType, MetricsType, SGDOptimizer
from flexflow.keras.datasets import cifar10
from flexflow.torch.model import file_to_ff


def top_level_task():
    path = ff_path("cnn.ff")
    if not os.path.exists(path):
        from cifar10_cnn_torch import export
        export(path)
    ffconfig = FFConfig()
    ffconfig.parse_args()
    m = FFModel(ffconfig)
    x = m.create_tensor([ffconfig.batch_size, 3, 32, 32], DataType.DT_FLOAT)
    outs = file_to_ff(path, m, [x, x])
    m.softmax(outs[0])
    m.optimizer = SGDOptimizer(m, 0.01)
    m.compile(loss_type=LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY,
              metrics=[MetricsType.METRICS_ACCURACY, MetricsType.METRICS_SPARSE_CATEGORICAL_CROSSENTROPY])
    (xt, yt), _ = cifar10.load_data(num_samples(10000))
    dl_x = m.create_data_loader(x, xt.astype("float32") / 255)
    dl_y = m.create_data_loader(m.label_tensor, yt.astype("int32"))
    m.init_layers()
    for layer in m.get_layers():
        print(layer.name)
    ts = ffconfig.get_current_time()
    m.fit(x=dl_x, y=dl_y, epochs=ffconfig.epochs)
    report(ffconfig, ts, dl_x.num_samples, ffconfig.epochs)


if __name__ == "__main__":
    print("cifar10 cnn")
    top_level_task()
