"""flexflow.onnx (reference: python/flexflow/onnx/model.py)."""
from flexflow_train_amd.frontends.onnx import (ONNXModel, ONNXModelKeras, encode_model, export_keras,  # noqa: F401
                                               export_torch)
