"""Attach a numpy array to an input tensor and read it back (reference:
examples/python/native/tensor_attach.py)."""
import numpy as np
import _common  # noqa: F401

from flexflow.core import DataType, FFConfig, FFModel, NetConfig


def top_level_task():
    ffconfig = FFConfig()
    ffconfig.parse_args()
    print(NetConfig().dataset_path)
    m = FFModel(ffconfig)
    inp = m.create_tensor([8, 3, 10, 10], DataType.DT_FLOAT)
    arr = np.arange(8 * 3 * 10 * 10, dtype=np.float32).reshape(8, 3, 10, 10)
    inp.attach_numpy_array(ffconfig, arr)
    out = inp.get_array(ffconfig, DataType.DT_FLOAT)
    print(out.shape, out.ravel()[:5])
    assert np.array_equal(out, arr)
    inp.detach_numpy_array(ffconfig)
    print("THROUGHPUT = n/a (tensor attach only)")


if __name__ == "__main__":
    print("tensor attach")
    top_level_task()
