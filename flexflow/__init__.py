"""``flexflow`` compatibility namespace: the reference's Python API
(python/flexflow/{core,torch,keras,onnx}) on top of flexflow_train_amd."""
