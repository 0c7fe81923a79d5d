"""CIFAR-10 CNN trained by an explicit loop that attaches every batch with
set_tensor (reference: examples/python/native/cifar10_cnn_attach.py)."""
from _common import num_samples, report

from flexflow.core import ActiMode, DataType, FFConfig, FFModel, LossType, MetricsType, NetConfig, SGDOptimizer
from flexflow.keras.datasets import cifar10


def next_batch(idx, data, tensor, ffconfig, ffmodel):
    start = idx * ffconfig.batch_size
    tensor.set_tensor(ffmodel, data[start:start + ffconfig.batch_size])


def top_level_task():
    ffconfig = FFConfig()
    ffconfig.parse_args()
    print(NetConfig().dataset_path)
    m = FFModel(ffconfig)
    x = m.create_tensor([ffconfig.batch_size, 3, 32, 32], DataType.DT_FLOAT)
    R = ActiMode.AC_MODE_RELU
    t = m.conv2d(x, 32, 3, 3, 1, 1, 1, 1, R)
    t = m.conv2d(t, 32, 3, 3, 1, 1, 1, 1, R)
    t = m.pool2d(t, 2, 2, 2, 2, 0, 0)
    t = m.conv2d(t, 64, 3, 3, 1, 1, 1, 1, R)
    t = m.conv2d(t, 64, 3, 3, 1, 1, 1, 1, R)
    t = m.pool2d(t, 2, 2, 2, 2, 0, 0)
    t = m.flat(t)
    t = m.dense(t, 512, R)
    t = m.softmax(m.dense(t, 10))
    m.optimizer = SGDOptimizer(m, 0.01)
    m.compile(loss_type=LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY,
              metrics=[MetricsType.METRICS_ACCURACY, MetricsType.METRICS_SPARSE_CATEGORICAL_CROSSENTROPY])
    n = num_samples(10000)
    (xt, yt), _ = cifar10.load_data(n)
    xt, yt = xt.astype("float32") / 255, yt.astype("int32")
    label = m.label_tensor
    next_batch(0, xt, x, ffconfig, m)
    next_batch(0, yt, label, ffconfig, m)
    m.init_layers()
    ts = ffconfig.get_current_time()
    for _ in range(ffconfig.epochs):
        m.reset_metrics()
        for it in range(n // ffconfig.batch_size):
            next_batch(it, xt, x, ffconfig, m)
            next_batch(it, yt, label, ffconfig, m)
            m.forward()
            m.zero_gradients()
            m.backward()
            m.update()
    report(ffconfig, ts, n, ffconfig.epochs)
    print(m.get_perf_metrics())


if __name__ == "__main__":
    print("cifar10 cnn attach")
    top_level_task()
