"""User-facing frontends: PyTorch (torch.fx + .ff IR), Keras-style, ONNX."""
