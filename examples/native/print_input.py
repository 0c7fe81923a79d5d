"""Map input tensors as host arrays, write into them, and read a layer's
input tensor back (reference: examples/python/native/print_input.py)."""
import numpy as np
import _common  # noqa: F401

from flexflow.core import ActiMode, DataType, FFConfig, FFModel


def top_level_task():
    ffconfig = FFConfig()
    ffconfig.parse_args()
    m = FFModel(ffconfig)
    input1 = m.create_tensor([ffconfig.batch_size, 3, 229, 229], DataType.DT_FLOAT)
    input2 = m.create_tensor([ffconfig.batch_size, 256], DataType.DT_FLOAT)
    input1.inline_map(ffconfig)
    a1 = input1.get_array(ffconfig)
    print(hex(a1.__array_interface__["data"][0]), a1.shape)
    input1.inline_unmap(ffconfig)
    input2.inline_map(ffconfig)
    a2 = input2.get_array(ffconfig)
    a2 *= 0
    a2 += 2.2
    input2.inline_unmap(ffconfig)
    m.conv2d(input1, 64, 11, 11, 4, 4, 2, 2)
    t = m.dense(input2, 128, ActiMode.AC_MODE_RELU)
    m.dense(t, 128, ActiMode.AC_MODE_RELU)
    dense1 = m.get_layer_by_id(1)
    t2 = dense1.get_input_tensor()
    t2.inline_map(ffconfig)
    a22 = t2.get_array(ffconfig)
    print(a22.shape, a22.ravel()[:4])
    t2.inline_unmap(ffconfig)
    assert np.allclose(a22, 2.2)
    print("THROUGHPUT = n/a (tensor inspection only)")


if __name__ == "__main__":
    print("print input")
    top_level_task()
