"""Teacher -> student weight transfer on a Sequential CNN (reference:
examples/python/keras/seq_mnist_cnn_net2net.py)."""
from _common import ModelAccuracy, epochs, mnist_images, verify

import flexflow.keras.optimizers
from flexflow.keras.layers import Activation, Conv2D, Dense, Flatten, MaxPooling2D
from flexflow.keras.models import Sequential


def build(dense1_name=None):
    model = Sequential()
    model.add(Conv2D(filters=32, input_shape=(1, 28, 28), kernel_size=(3, 3), strides=(1, 1), padding=(1, 1),
                     activation="relu"))
    model.add(Conv2D(filters=64, kernel_size=(3, 3), strides=(1, 1), padding=(1, 1), activation="relu"))
    model.add(MaxPooling2D(pool_size=(2, 2), strides=(2, 2), padding="valid"))
    model.add(Flatten())
    model.add(Dense(128, activation="relu", name=dense1_name))
    model.add(Dense(10))
    model.add(Activation("softmax"))
    model.compile(optimizer=flexflow.keras.optimizers.SGD(learning_rate=0.01), loss="sparse_categorical_crossentropy",
                  metrics=["accuracy", "sparse_categorical_crossentropy"])
    return model


def top_level_task():
    x_train, y_train = mnist_images()
    teacher = build()
    teacher.fit(x_train, y_train, epochs=epochs(5))
    w = {i: teacher.get_layer(index=i).get_weights(teacher.ffmodel) for i in (0, 1, 4, 5)}
    student = build("dense1")
    for i in (0, 1, 5):
        student.get_layer(index=i).set_weights(student.ffmodel, *w[i])
    student.get_layer(name="dense1").set_weights(student.ffmodel, *w[4])
    print(student.summary())
    student.fit(x_train, y_train, epochs=epochs(5), callbacks=verify(ModelAccuracy.MNIST_CNN))


if __name__ == "__main__":
    print("Sequential model, mnist cnn teacher student")
    top_level_task()
