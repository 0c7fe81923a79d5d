from flexflow_train_amd.frontends.onnx import *  # noqa: F401,F403
from flexflow_train_amd.frontends.onnx import (ONNXModel, ONNXModelKeras, encode_model, export_keras,  # noqa: F401
                                               export_torch)
