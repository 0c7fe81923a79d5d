"""Teacher -> student weight transfer with get_weights / set_weights on a
functional MLP (reference: examples/python/keras/func_mnist_mlp_net2net.py)."""
from _common import ModelAccuracy, epochs, mnist_flat, verify

import flexflow.keras.optimizers
from flexflow.keras.layers import Activation, Dense, Input
from flexflow.keras.models import Model


def build(names=("dense1", "dense2", "dense3")):
    inp = Input(shape=(784,))
    t = Dense(512, input_shape=(784,), activation="relu", name=names[0])(inp)
    t = Dense(512, activation="relu", name=names[1])(t)
    t = Dense(10, name=names[2])(t)
    model = Model(inp, Activation("softmax")(t))
    model.compile(optimizer=flexflow.keras.optimizers.SGD(learning_rate=0.01), loss="sparse_categorical_crossentropy",
                  metrics=["accuracy", "sparse_categorical_crossentropy"])
    return model


def top_level_task():
    x_train, y_train = mnist_flat()
    teacher = build()
    teacher.fit(x_train, y_train, epochs=epochs(10))
    weights = [teacher.get_layer(index=i).get_weights(teacher.ffmodel) for i in range(3)]
    student = build(("s_dense1", "s_dense2", "s_dense3"))
    for i, (k, b) in enumerate(weights):
        student.get_layer(index=i).set_weights(student.ffmodel, k, b)
    print(student.summary())
    student.fit(x_train, y_train, epochs=epochs(10), callbacks=verify(ModelAccuracy.MNIST_MLP))


if __name__ == "__main__":
    print("Functional API, mnist mlp teacher student")
    top_level_task()
