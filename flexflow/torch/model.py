from flexflow_train_amd.frontends.torch_fx import *  # noqa: F401,F403
from flexflow_train_amd.frontends.torch_fx import (IR_DELIMITER, INOUT_NODE_DELIMITER,  # noqa: F401
                                                   PyTorchModel, copy_weights, string_to_ff)


def file_to_ff(filename, ffmodel, input_tensors):
    return PyTorchModel.file_to_ff(filename, ffmodel, input_tensors)
