"""Export the MNIST MLP from the keras frontend to mnist_mlp_keras.onnx
(reference: examples/python/onnx/mnist_mlp_keras.py, which uses keras2onnx)."""
from _common import onnx_path

from flexflow.keras.layers import Activation, Dense, Input
from flexflow.keras.models import Model
from flexflow.onnx.model import ONNXModel, export_keras


def export(path=None):
    path = path or onnx_path("mnist_mlp_keras.onnx")
    inp = Input(shape=(784,))
    t = Dense(512, activation="relu")(inp)
    t = Dense(512, activation="relu")(t)
    t = Dense(10)(t)
    model = Model(inp, Activation("softmax")(t))
    model.compile(optimizer="sgd", loss="sparse_categorical_crossentropy", metrics=["accuracy"])
    export_keras(model, path)
    return path


if __name__ == "__main__":
    p = export()
    for node in ONNXModel(p).graph.nodes:
        print(node.op_type, node.inputs, node.outputs)
