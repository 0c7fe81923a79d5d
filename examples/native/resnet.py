"""ResNet-50 on CIFAR-10 images upsampled to 229x229 through the native API
(reference: examples/python/native/resnet.py; network as
flexflow_train_amd/models/cnn.py build_resnet50)."""
import numpy as np
from _common import num_samples, report

from flexflow.core import FFConfig, FFModel, LossType, MetricsType, SGDOptimizer
from flexflow.keras.datasets import cifar10
from flexflow_train_amd.models.cnn import CNNConfig, build_resnet50


def top_level_task():
    ffconfig = FFConfig()
    ffconfig.parse_args()
    m = FFModel(ffconfig)
    build_resnet50(m, CNNConfig(batch_size=ffconfig.batch_size, image_size=229, num_classes=10))
    m.optimizer = SGDOptimizer(m, 0.001)
    m.compile(loss_type=LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY,
              metrics=[MetricsType.METRICS_ACCURACY, MetricsType.METRICS_SPARSE_CATEGORICAL_CROSSENTROPY])
    (x, y), _ = cifar10.load_data(num_samples(10000))
    idx = np.arange(229) * 32 // 229
    x = x[:, :, idx][:, :, :, idx].astype("float32") / 255
    ts = ffconfig.get_current_time()
    m.fit(x=x, y=y.astype("int32"), epochs=ffconfig.epochs)
    report(ffconfig, ts, len(x), ffconfig.epochs)


if __name__ == "__main__":
    print("resnet")
    top_level_task()
