"""Reuters topic classification MLP on a binary bag-of-words (reference:
examples/python/keras/seq_reuters_mlp.py)."""
import numpy as np
from _common import ModelAccuracy, epochs, num_samples, verify

import flexflow.keras.optimizers
from flexflow.keras.datasets import reuters
from flexflow.keras.layers import Activation, Dense, Input
from flexflow.keras.models import Sequential
from flexflow.keras.preprocessing.text import Tokenizer


def top_level_task():
    max_words = 1000
    (x_train, y_train), (x_test, y_test) = reuters.load_data(num_words=max_words, test_split=0.2)
    n = min(len(x_train), num_samples(len(x_train)))
    x_train, y_train = x_train[:n], y_train[:n]
    num_classes = int(np.max(y_train)) + 1
    tokenizer = Tokenizer(num_words=max_words)
    x_train = tokenizer.sequences_to_matrix(x_train, mode="binary").astype("float32")
    y_train = np.reshape(y_train.astype("int32"), (len(y_train), 1))
    print("x_train shape:", x_train.shape, "classes:", num_classes)
    model = Sequential()
    model.add(Input(shape=(max_words,)))
    model.add(Dense(512, activation="relu"))
    model.add(Dense(num_classes))
    model.add(Activation("softmax"))
    model.compile(optimizer=flexflow.keras.optimizers.Adam(learning_rate=0.01), loss="sparse_categorical_crossentropy",
                  metrics=["accuracy", "sparse_categorical_crossentropy"])
    print(model.summary())
    model.fit(x_train, y_train, epochs=epochs(5), callbacks=verify(ModelAccuracy.REUTERS_MLP))


if __name__ == "__main__":
    print("Sequential model, reuters mlp")
    top_level_task()
