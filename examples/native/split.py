"""Concat of three conv towers split back into three, training on one
piece (reference: examples/python/native/split.py)."""
from _common import num_samples, report

from flexflow.core import (ActiMode, DataType, FFConfig, FFModel, LossType, MetricsType, NetConfig, PoolType,
                           SGDOptimizer)
from flexflow.keras.datasets import cifar10


def top_level_task():
    ffconfig = FFConfig()
    ffconfig.parse_args()
    print(NetConfig().dataset_path)
    m = FFModel(ffconfig)
    x = m.create_tensor([ffconfig.batch_size, 3, 32, 32], DataType.DT_FLOAT)
    R = ActiMode.AC_MODE_RELU
    towers = [m.conv2d(x, 32, 3, 3, 1, 1, 1, 1, R) for _ in range(3)]
    ts_ = m.split(m.concat(towers, 1), 3, 1)
    t = m.conv2d(ts_[1], 32, 3, 3, 1, 1, 1, 1, R)
    t = m.pool2d(t, 2, 2, 2, 2, 0, 0)
    t = m.conv2d(t, 64, 3, 3, 1, 1, 1, 1, R)
    t = m.conv2d(t, 64, 3, 3, 1, 1, 1, 1, R)
    t = m.pool2d(t, 2, 2, 2, 2, 0, 0, PoolType.POOL_MAX)
    t = m.flat(t)
    t = m.dense(t, 512, R)
    t = m.softmax(m.dense(t, 10))
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
    print("cifar10 cnn split")
    top_level_task()
