"""AlexNet on CIFAR-10 images upsampled to 229x229 through the native API
(reference: examples/python/native/alexnet.py; network as
flexflow_train_amd/models/cnn.py build_alexnet)."""
import numpy as np
from _common import num_samples, report

from flexflow.core import FFConfig, FFModel, LossType, MetricsType, SGDOptimizer
from flexflow.keras.datasets import cifar10
from flexflow_train_amd.models.cnn import CNNConfig, build_alexnet


def top_level_task():
    ffconfig = FFConfig()
    ffconfig.parse_args()
    print("Python API batchSize(%d) workersPerNodes(%d) numNodes(%d)" %
          (ffconfig.batch_size, ffconfig.workers_per_node, ffconfig.num_nodes))
    m = FFModel(ffconfig)
    build_alexnet(m, CNNConfig(batch_size=ffconfig.batch_size, image_size=229, num_classes=10, batch_norm=False))
    m.optimizer = SGDOptimizer(m, 0.01)
    m.compile(loss_type=LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY,
              metrics=[MetricsType.METRICS_ACCURACY, MetricsType.METRICS_SPARSE_CATEGORICAL_CROSSENTROPY])
    (x, y), _ = cifar10.load_data(num_samples(10000))
    idx = (np.arange(229) * 32 // 229)
    x = x[:, :, idx][:, :, :, idx].astype("float32") / 255          # nearest-neighbour resize
    dl_x = m.create_data_loader(m._inputs[0], x)
    dl_y = m.create_data_loader(m.label_tensor, y.astype("int32"))
    m.init_layers()
    ts = ffconfig.get_current_time()
    m.fit(x=dl_x, y=dl_y, epochs=ffconfig.epochs)
    report(ffconfig, ts, len(x), ffconfig.epochs)


if __name__ == "__main__":
    print("alexnet")
    top_level_task()
