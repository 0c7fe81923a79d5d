"""Loss functions and training metrics.

Parity: lib/kernels/src/cuda/loss_function_kernels.cu (sparse CCE: grad =
softmax - onehot; CCE: p - y; MSE; identity; all scaled by 1/batch, :21-137),
lib/kernels/src/cuda/metrics_functions.cu (accuracy / CCE / sparse CCE / MSE
/ RMSE / MAE accumulated on the device with atomics, :23-185),
lib/kernels/include/kernels/perf_metrics.h (PerfMetrics).

As in the reference the (sparse) cross-entropy losses consume the logits of a
trailing SOFTMAX (the executor fuses softmax + CE, whose backward the
reference expresses as a copy, softmax_kernels.cu:63-72): on GPU one HIP
kernel computes loss, gradient (in place over the logits), and metrics.
Metrics accumulate in a small device buffer and are read on demand, so the
training loop never synchronises with the host.
"""
from __future__ import annotations

import dataclasses
import math
import time
from typing import Optional

import torch

from .. import kernels as K

LOSS_TYPES = ("categorical_crossentropy", "sparse_categorical_crossentropy", "mean_squared_error",
              "mean_squared_error_sum", "identity")

# device metric slots
M_LOSS, M_CORRECT, M_COUNT, M_SQERR, M_ABSERR, M_CCE = 0, 1, 2, 3, 4, 5
N_SLOTS = 8


def normalize_loss_type(t) -> str:
    s = str(getattr(t, "name", t)).lower()
    s = s.replace("loss_", "")
    aliases = {
        "sparse_categorical_crossentropy": "sparse_categorical_crossentropy",
        "categorical_crossentropy": "categorical_crossentropy",
        "mean_squared_error_avg_reduce": "mean_squared_error",
        "mean_squared_error": "mean_squared_error",
        "mse": "mean_squared_error",
        "mean_squared_error_sum_reduce": "mean_squared_error_sum",
        "identity": "identity",
    }
    if s not in aliases:
        raise ValueError(f"unknown loss type {t}")
    return aliases[s]


class LossFunction:
    def __init__(self, loss_type, global_rows: int, valid_cols: Optional[int] = None):
        self.loss_type = normalize_loss_type(loss_type)
        self.global_rows = global_rows
        self.valid_cols = valid_cols

    @property
    def fuses_softmax(self) -> bool:
        return self.loss_type in ("categorical_crossentropy", "sparse_categorical_crossentropy")

    def __call__(self, logits: torch.Tensor, labels: torch.Tensor, metrics: torch.Tensor) -> torch.Tensor:
        """Returns d(loss)/d(logits) for the LOCAL piece; the loss is the mean
        over the GLOBAL batch (gradients are later summed across DP ranks)."""
        lt = self.loss_type
        C = logits.shape[-1]
        rows = logits.numel() // C
        scale = 1.0 / self.global_rows
        if lt == "sparse_categorical_crossentropy":
            lab = labels.reshape(-1)
            if lab.dtype not in (torch.int32, torch.int64):
                lab = lab.long()
            if logits.is_cuda and K.available() and logits.dtype in (torch.bfloat16, torch.float32):
                g = logits.contiguous().view(rows, C)
                K.softmax_ce(g, lab.contiguous(), scale, metrics=metrics, valid_cols=self.valid_cols)
                return g.view(logits.shape)
            lf = logits.reshape(rows, C).float()
            if self.valid_cols is not None and self.valid_cols < C:
                lf = lf.clone()
                lf[:, self.valid_cols:] = float("-inf")
            lse = torch.logsumexp(lf, -1)
            lab64 = lab.long()
            # labels outside [0, C) (e.g. -100 padding) are ignored, as in the
            # HIP kernel: no loss, no gradient, not counted
            valid = (lab64 >= 0) & (lab64 < C)
            safe = torch.where(valid, lab64, torch.zeros_like(lab64))
            ll = lf.gather(1, safe.view(-1, 1)).view(-1)
            vf = valid.float()
            metrics[M_LOSS] += ((lse - ll) * vf).sum()
            metrics[M_CORRECT] += ((lf.argmax(-1) == lab64).float() * vf).sum()
            metrics[M_COUNT] += vf.sum()
            p = torch.softmax(lf, -1)
            p[torch.arange(rows, device=p.device), safe] -= vf
            p *= vf.view(-1, 1)
            return (p * scale).to(logits.dtype).view(logits.shape)
        if lt == "categorical_crossentropy":
            lf = logits.reshape(rows, C).float()
            y = labels.reshape(rows, C).float()
            lsm = torch.log_softmax(lf, -1)
            metrics[M_LOSS] += -(y * lsm).sum()
            metrics[M_CORRECT] += (lf.argmax(-1) == y.argmax(-1)).float().sum()
            metrics[M_COUNT] += rows
            return ((torch.softmax(lf, -1) - y) * scale).to(logits.dtype).view(logits.shape)
        if lt in ("mean_squared_error", "mean_squared_error_sum"):
            s = (2.0 / (self.global_rows * C)) if lt == "mean_squared_error" else 2.0
            y = labels.reshape(logits.shape)
            if (K.tensorop_ok(logits) and metrics.dtype == torch.float32 and metrics.is_cuda
                    and metrics.is_contiguous() and logits.numel() > 0):
                # one HIP pass: the gradient and every metric slot (loss,
                # count, squared / absolute error); fp32 labels read as they are
                if y.dtype not in (logits.dtype, torch.float32):
                    y = y.float()
                g = torch.empty_like(logits)
                K.mse_full(logits.contiguous(), y.contiguous(), g, metrics, s, C, rows)
                return g
            p = logits.float()
            y = labels.reshape(p.shape).float()
            d = p - y
            metrics[M_SQERR] += (d * d).sum()
            metrics[M_ABSERR] += d.abs().sum()
            metrics[M_LOSS] += (d * d).sum() / C
            metrics[M_COUNT] += rows
            return (d * s).to(logits.dtype)
        # identity: the output itself is the loss
        metrics[M_LOSS] += logits.float().sum()
        metrics[M_COUNT] += rows
        return torch.full_like(logits, scale)


_METRIC_NAMES = {
    "accuracy": "accuracy", "metrics_accuracy": "accuracy",
    "categorical_crossentropy": "categorical_crossentropy",
    "metrics_categorical_crossentropy": "categorical_crossentropy",
    "sparse_categorical_crossentropy": "sparse_categorical_crossentropy",
    "metrics_sparse_categorical_crossentropy": "sparse_categorical_crossentropy",
    "mean_squared_error": "mean_squared_error", "metrics_mean_squared_error": "mean_squared_error", "mse": "mean_squared_error",
    "root_mean_squared_error": "root_mean_squared_error", "metrics_root_mean_squared_error": "root_mean_squared_error",
    "mean_absolute_error": "mean_absolute_error", "metrics_mean_absolute_error": "mean_absolute_error",
}


def normalize_metric(m) -> str:
    s = str(getattr(m, "name", m)).lower()
    if s not in _METRIC_NAMES:
        raise ValueError(f"unknown metric {m}")
    return _METRIC_NAMES[s]


@dataclasses.dataclass
class PerfMetrics:
    """Host view of the accumulated metrics (perf_metrics.h:9-92)."""

    train_all: int = 0
    train_correct: int = 0
    cce_loss: float = 0.0
    sparse_cce_loss: float = 0.0
    mse_loss: float = 0.0
    rmse_loss: float = 0.0
    mae_loss: float = 0.0
    loss: float = 0.0
    start_time: float = dataclasses.field(default_factory=time.time)
    current_time: float = dataclasses.field(default_factory=time.time)
    metrics: tuple = ()

    @property
    def accuracy(self) -> float:
        return self.train_correct / self.train_all if self.train_all else 0.0

    def get_accuracy(self) -> float:
        """Percent, as the reference's PerfMetrics.get_accuracy (flexflow_cffi.py)."""
        return 100.0 * self.accuracy

    @classmethod
    def from_buffer(cls, buf: torch.Tensor, metrics, loss_type: str, start_time: float, out_dim: int = 1):
        v = buf.detach().double().cpu().tolist()
        n = max(1.0, v[M_COUNT])
        pm = cls(train_all=int(v[M_COUNT]), train_correct=int(v[M_CORRECT]), start_time=start_time,
                 current_time=time.time(), metrics=tuple(metrics))
        pm.loss = v[M_LOSS] / n
        if loss_type == "sparse_categorical_crossentropy":
            pm.sparse_cce_loss = pm.loss
        if loss_type == "categorical_crossentropy":
            pm.cce_loss = pm.loss
        pm.mse_loss = v[M_SQERR] / (n * max(1, out_dim))
        pm.rmse_loss = math.sqrt(max(pm.mse_loss, 0.0))
        pm.mae_loss = v[M_ABSERR] / (n * max(1, out_dim))
        return pm


    def get_throughput(self) -> float:
        return self.train_all / max(1e-9, self.current_time - self.start_time)

    def __str__(self):
        parts = [f"samples={self.train_all}"]
        if "accuracy" in self.metrics:
            parts.append(f"accuracy={self.get_accuracy():.2f}%")
        for m, v in (("sparse_categorical_crossentropy", self.sparse_cce_loss),
                     ("categorical_crossentropy", self.cce_loss), ("mean_squared_error", self.mse_loss),
                     ("root_mean_squared_error", self.rmse_loss), ("mean_absolute_error", self.mae_loss)):
            if m in self.metrics:
                parts.append(f"{m}={v:.4f}")
        parts.append(f"loss={self.loss:.4f}")
        return " ".join(parts)
