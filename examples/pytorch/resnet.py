"""Rebuild ResNet-18 from resnet18.ff and evaluate it on CIFAR-10 upsampled
to 224x224 (reference: examples/python/pytorch/resnet.py)."""
import os

from _common import ff_path, num_samples, report, upsample

from flexflow.core import DataType, FFConfig, FFModel, LossType, MetricsType, NetConfig, SGDOptimizer
from flexflow.keras.datasets import cifar10
from flexflow.torch.model import PyTorchModel


def top_level_task():
    path = ff_path("resnet18.ff")
    if not os.path.exists(path):
        from resnet_torch import export
        export(path)
    ffconfig = FFConfig()
    ffconfig.parse_args()
    print(NetConfig().dataset_path)
    m = FFModel(ffconfig)
    x = m.create_tensor([ffconfig.batch_size, 3, 224, 224], DataType.DT_FLOAT)
    outs = PyTorchModel.file_to_ff(path, m, [x])
    m.softmax(outs[0])
    m.optimizer = SGDOptimizer(m, 0.01)
    m.compile(loss_type=LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY,
              metrics=[MetricsType.METRICS_ACCURACY, MetricsType.METRICS_SPARSE_CATEGORICAL_CROSSENTROPY])
    (xt, yt), _ = cifar10.load_data(num_samples(10000))
    dl_x = m.create_data_loader(x, upsample(xt, 224).astype("float32") / 255)
    dl_y = m.create_data_loader(m.label_tensor, yt.astype("int32"))
    assert dl_x.num_samples == dl_y.num_samples
    m.init_layers()
    ts = ffconfig.get_current_time()
    m.eval(x=dl_x, y=dl_y)
    report(ffconfig, ts, dl_x.num_samples, 1)


if __name__ == "__main__":
    print("resnet18 (torch -> .ff)")
    top_level_task()
