"""Keras callbacks (reference: python/flexflow/keras/callbacks.py)."""
from __future__ import annotations


class Callback:
    def __init__(self):
        self.model = None
        self.params = {}

    def set_params(self, params):
        self.params = params

    def set_model(self, model):
        self.model = model

    def on_epoch_begin(self, epoch, logs=None): ...

    def on_epoch_end(self, epoch, logs=None): ...

    def on_batch_begin(self, batch, logs=None): ...

    def on_batch_end(self, batch, logs=None): ...

    def on_train_begin(self, logs=None): ...

    def on_train_end(self, logs=None): ...


class LearningRateScheduler(Callback):
    """lr = schedule(epoch) at the start of every epoch."""

    def __init__(self, schedule):
        super().__init__()
        self.schedule = schedule

    def on_epoch_begin(self, epoch, logs=None):
        lr = float(self.schedule(epoch))
        self.model.optimizer.set_learning_rate(lr)
        print(f"set learning rate {lr}")


def _accuracy(model) -> float:
    return model.ffmodel.get_perf_metrics().get_accuracy()   # percent


class VerifyMetrics(Callback):
    """Fails the run (AssertionError) when the final accuracy (percent) is
    below ``accuracy`` (the reference's CI examples use it)."""

    def __init__(self, accuracy):
        super().__init__()
        self.accuracy = float(getattr(accuracy, "value", accuracy))

    def on_train_end(self, logs=None):
        acc = _accuracy(self.model)
        assert acc >= self.accuracy, f"Accuracy check failed: {acc:.2f}% < {self.accuracy}%"
        print(f"Accuracy check passed: {acc:.2f}% >= {self.accuracy}%")


class EpochVerifyMetrics(Callback):
    """Stops training early (on_epoch_end returns True) once the accuracy
    reaches ``accuracy`` percent."""

    def __init__(self, accuracy, early_stop=True):
        super().__init__()
        self.accuracy = float(getattr(accuracy, "value", accuracy))
        self.early_stop = early_stop

    def on_epoch_end(self, epoch, logs=None):
        return bool(self.early_stop and _accuracy(self.model) >= self.accuracy)
