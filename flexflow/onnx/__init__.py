"""flexflow.onnx (reference: python/flexflow/onnx/model.py)."""
from flexflow_train_amd.frontends.onnx import ONNXModel, encode_model  # noqa: F401
