"""Backend layers used by the keras backend functions (reference:
python/flexflow/keras/backend/internal.py)."""
from __future__ import annotations

from ..layers import Layer


class BatchMatmul(Layer):
    """(…, M, K) x (…, K, N) -> (…, M, N)."""

    def out_shape(self, s):
        a, b = s
        if a[-1] != b[-2]:
            raise ValueError(f"batch_dot: inner dims differ {a} x {b}")
        return a[:-1] + (b[-1],)

    def build_ff(self, ff, ins):
        return ff.batch_matmul(ins[0], ins[1], name=self.name)


class _Unary(Layer):
    fn = ""

    def build_ff(self, ff, ins):
        return getattr(ff, self.fn)(ins[0], name=self.name)


class Sin(_Unary):
    fn = "sin"


class Cos(_Unary):
    fn = "cos"


class Exp(_Unary):
    fn = "exp"


class Rsqrt(_Unary):
    fn = "rsqrt"


class Pow(Layer):
    def __init__(self, a, name=None):
        super().__init__(name)
        self.a = float(a)

    def build_ff(self, ff, ins):
        return ff.pow(ins[0], self.a, name=self.name)


class ReduceSum(Layer):
    """Sum over ``axis`` (axes count the batch dimension, as in the
    reference: sum(x, axis=1) on (B, N) gives (B,))."""

    def __init__(self, axis=None, keepdims=False, name=None):
        super().__init__(name)
        self.axis, self.keepdims = axis, keepdims

    def _axes(self, nd):
        if self.axis is None:
            return list(range(1, nd))
        ax = self.axis if isinstance(self.axis, (list, tuple)) else [self.axis]
        return sorted(a % nd for a in ax)

    def out_shape(self, s):
        axes = self._axes(len(s[0]))
        if self.keepdims:
            return tuple(1 if i in axes else d for i, d in enumerate(s[0]))
        return tuple(d for i, d in enumerate(s[0]) if i not in axes)

    def build_ff(self, ff, ins):
        return ff.reduce_sum(ins[0], self._axes(len(ins[0].dims)), self.keepdims, name=self.name)


class Gather(Layer):
    """torch.gather along ``axis``: out[i][j][k] = x[i][idx[i][j][k]][k]
    (axis 1), output shaped like the index."""

    def __init__(self, axis, name=None):
        super().__init__(name)
        self.axis = axis

    def out_shape(self, s):
        return s[1]

    def out_dtype(self, dtypes):
        return dtypes[0]

    def build_ff(self, ff, ins):
        return ff.gather(ins[0], ins[1], self.axis, name=self.name)


def batch_dot(x, y):
    return BatchMatmul()([x, y])


def sin(x):
    return Sin()(x)


def cos(x):
    return Cos()(x)


def exp(x):
    return Exp()(x)


def pow(x, a):  # noqa: A001
    return Pow(a)(x)


def sum(x, axis=None, keepdims=False):  # noqa: A001
    return ReduceSum(axis, keepdims)(x)


def rsqrt(x):
    return Rsqrt()(x)


def gather(x, indices, axis):
    return Gather(axis)([x, indices])
