"""Trigonometric and hyperbolic functions (reference ``heat/core/trigonometrics.py``)."""
from __future__ import annotations

import math

import torch

from . import _operations
from .dndarray import DNDarray

__all__ = ["acos", "acosh", "asin", "asinh", "atan", "atan2", "atanh", "arccos", "arccosh", "arcsin",
           "arcsinh", "arctan", "arctan2", "arctanh", "cos", "cosh", "deg2rad", "degrees", "rad2deg",
           "radians", "sin", "sinh", "tan", "tanh"]


def _u(fn):
    def f(x, out=None):
        return _operations.local_op(fn, x, out)

    f.__doc__ = "Element-wise {} (integers are promoted to floating point).".format(fn.__name__)
    return f


acos = arccos = _u(torch.acos)
acosh = arccosh = _u(torch.acosh)
asin = arcsin = _u(torch.asin)
asinh = arcsinh = _u(torch.asinh)
atan = arctan = _u(torch.atan)
atanh = arctanh = _u(torch.atanh)
cos = _u(torch.cos)
cosh = _u(torch.cosh)
sin = _u(torch.sin)
sinh = _u(torch.sinh)
tan = _u(torch.tan)
tanh = _u(torch.tanh)
deg2rad = radians = _u(torch.deg2rad)
rad2deg = degrees = _u(torch.rad2deg)


def arctan2(x1, x2, out=None) -> DNDarray:
    """Element-wise arc tangent of x1/x2 choosing the quadrant correctly."""
    def _atan2(a, b):
        # exact types promote like the reference's local ops: int64 -> float64, others -> float32
        if not a.is_floating_point():
            a = a.double() if a.dtype == torch.int64 else a.float()
        if not b.is_floating_point():
            b = b.double() if b.dtype == torch.int64 else b.float()
        return torch.atan2(a, b)

    return _operations.binary_op(_atan2, x1, x2, out)


atan2 = arctan2

for _n in ("acos", "acosh", "asin", "asinh", "atan", "atanh", "cos", "cosh", "sin", "sinh", "tan", "tanh",
           "arccos", "arcsin", "arctan", "arccosh", "arcsinh", "arctanh"):
    setattr(DNDarray, _n, (lambda f: lambda self, out=None: f(self, out))(globals()[_n]))
DNDarray.atan2 = lambda self, other, out=None: arctan2(self, other, out)
