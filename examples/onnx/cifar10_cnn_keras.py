"""Export the CIFAR-10 CNN from the keras frontend to cifar10_cnn_keras.onnx
(reference: examples/python/onnx/cifar10_cnn_keras.py, keras2onnx)."""
from _common import onnx_path

from flexflow.keras.layers import Activation, Conv2D, Dense, Flatten, Input, MaxPooling2D
from flexflow.keras.models import Model
from flexflow.onnx.model import ONNXModel, export_keras


def export(path=None):
    path = path or onnx_path("cifar10_cnn_keras.onnx")
    inp = Input(shape=(3, 32, 32))
    t = Conv2D(filters=32, kernel_size=(3, 3), strides=(1, 1), padding="valid", activation="relu")(inp)
    t = Conv2D(filters=32, kernel_size=(3, 3), strides=(1, 1), padding="valid", activation="relu")(t)
    t = MaxPooling2D(pool_size=(2, 2), strides=(2, 2), padding="valid")(t)
    t = Conv2D(filters=64, kernel_size=(3, 3), strides=(1, 1), padding="valid", activation="relu")(t)
    t = Conv2D(filters=64, kernel_size=(3, 3), strides=(1, 1), padding="valid", activation="relu")(t)
    t = MaxPooling2D(pool_size=(2, 2), strides=(2, 2), padding="valid")(t)
    t = Flatten()(t)
    t = Dense(512, activation="relu")(t)
    t = Dense(10)(t)
    model = Model(inp, Activation("softmax")(t))
    print(model.summary())
    model.compile(optimizer="sgd", loss="sparse_categorical_crossentropy", metrics=["accuracy"])
    export_keras(model, path)
    return path


if __name__ == "__main__":
    for node in ONNXModel(export()).graph.nodes:
        print(node.op_type, node.inputs, node.outputs)
