from flexflow_train_amd.frontends.onnx import *  # noqa: F401,F403
from flexflow_train_amd.frontends.onnx import ONNXModel  # noqa: F401
