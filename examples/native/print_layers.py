"""Layer / parameter access: print the graph, overwrite a bias through its
Parameter, map the label tensor and edit it in place (reference:
examples/python/native/print_layers.py)."""
import numpy as np
import _common  # noqa: F401

from flexflow.core import ActiMode, DataType, FFConfig, FFModel, LossType, MetricsType, SGDOptimizer


def top_level_task():
    ffconfig = FFConfig()
    ffconfig.parse_args()
    print("Python API batchSize(%d) workersPerNodes(%d) numNodes(%d)" %
          (ffconfig.batch_size, ffconfig.workers_per_node, ffconfig.num_nodes))
    m = FFModel(ffconfig)
    input1 = m.create_tensor([ffconfig.batch_size, 3, 229, 229], DataType.DT_FLOAT)
    input2 = m.create_tensor([ffconfig.batch_size, 16], DataType.DT_FLOAT)
    m.conv2d(input1, 64, 11, 11, 4, 4, 2, 2)
    m.dense(input2, 8, ActiMode.AC_MODE_RELU)
    m.optimizer = SGDOptimizer(m, 0.01)
    m.compile(loss_type=LossType.LOSS_SPARSE_CATEGORICAL_CROSSENTROPY,
              metrics=[MetricsType.METRICS_ACCURACY, MetricsType.METRICS_SPARSE_CATEGORICAL_CROSSENTROPY])
    m.print_layers()
    label = m.label_tensor
    label.inline_map(m, ffconfig)
    arr = label.get_array(m, ffconfig)
    arr *= 0
    arr += 1
    print(arr.shape, arr.ravel()[:8])
    label.inline_unmap(m, ffconfig)
    assert (label.get_array(m, ffconfig) == 1).all()
    conv = m.get_layer_by_id(0)
    conv.get_bias_tensor().set_weights(m, np.full((64,), 22.222, np.float32))
    print(conv, conv.get_bias_tensor().get_weights(m)[:4])
    assert np.allclose(conv.get_bias_tensor().get_weights(m), 22.222)
    print("THROUGHPUT = n/a (layer inspection only)")


if __name__ == "__main__":
    print("print layers")
    top_level_task()
