"""Teacher -> student weight transfer on a Sequential MLP (reference:
examples/python/keras/seq_mnist_mlp_net2net.py)."""
from _common import ModelAccuracy, epochs, mnist_flat, verify

import flexflow.keras.optimizers
from flexflow.keras.layers import Activation, Dense
from flexflow.keras.models import Sequential


def build():
    model = Sequential()
    model.add(Dense(512, input_shape=(784,), activation="relu"))
    model.add(Dense(512, activation="relu"))
    model.add(Dense(10))
    model.add(Activation("softmax"))
    model.compile(optimizer=flexflow.keras.optimizers.SGD(learning_rate=0.01), loss="sparse_categorical_crossentropy",
                  metrics=["accuracy", "sparse_categorical_crossentropy"])
    return model


def top_level_task():
    x_train, y_train = mnist_flat()
    teacher = build()
    teacher.fit(x_train, y_train, epochs=epochs(10))
    student = build()
    for i in range(3):
        k, b = teacher.get_layer(index=i).get_weights(teacher.ffmodel)
        student.get_layer(index=i).set_weights(student.ffmodel, k, b)
    student.fit(x_train, y_train, epochs=epochs(10), callbacks=verify(ModelAccuracy.MNIST_MLP))


if __name__ == "__main__":
    print("Sequential model, mnist mlp teacher student")
    top_level_task()
