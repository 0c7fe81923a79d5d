"""CIFAR-10 CNN with two concatenated conv towers through the native API
(reference: examples/python/native/cifar10_cnn_concat.py)."""
from _common import num_samples, report

from flexflow.core import ActiMode, DataType, FFConfig, FFModel, LossType, MetricsType, PoolType, SGDOptimizer
from flexflow.keras.datasets import cifar10


def top_level_task():
    ffconfig = FFConfig()
    ffconfig.parse_args()
    m = FFModel(ffconfig)
    x = m.create_tensor([ffconfig.batch_size, 3, 32, 32], DataType.DT_FLOAT)
    R = ActiMode.AC_MODE_RELU
    t1 = m.conv2d(m.conv2d(x, 32, 3, 3, 1, 1, 1, 1, R), 32, 3, 3, 1, 1, 1, 1, R)
    t2 = m.conv2d(m.conv2d(x, 32, 3, 3, 1, 1, 1, 1, R), 32, 3, 3, 1, 1, 1, 1, R)
    t = m.concat([t1, t2], 1)
    t = m.pool2d(t, 2, 2, 2, 2, 0, 0, PoolType.POOL_MAX)
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
    ts = ffconfig.get_current_time()
    m.fit(x=xt.astype("float32") / 255, y=yt.astype("int32"), epochs=ffconfig.epochs)
    report(ffconfig, ts, len(xt), ffconfig.epochs)


if __name__ == "__main__":
    print("cifar10 cnn concat")
    top_level_task()
