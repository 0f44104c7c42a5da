"""Exponential and logarithmic functions (reference ``heat/core/exponential.py``)."""
from __future__ import annotations

import torch

from . import _operations
from .dndarray import DNDarray

__all__ = ["exp", "expm1", "exp2", "log", "log2", "log10", "log1p", "logaddexp", "logaddexp2", "sqrt", "square"]


def exp(x, out=None) -> DNDarray:
    return _operations.local_op(torch.exp, x, out)


def expm1(x, out=None) -> DNDarray:
    return _operations.local_op(torch.expm1, x, out)


def exp2(x, out=None) -> DNDarray:
    return _operations.local_op(torch.exp2, x, out)


def log(x, out=None) -> DNDarray:
    return _operations.local_op(torch.log, x, out)


def log2(x, out=None) -> DNDarray:
    return _operations.local_op(torch.log2, x, out)


def log10(x, out=None) -> DNDarray:
    return _operations.local_op(torch.log10, x, out)


def log1p(x, out=None) -> DNDarray:
    return _operations.local_op(torch.log1p, x, out)


def _floatify(a, b):
    if not (a.is_floating_point() or a.is_complex()):
        a = a.float()
    if not (b.is_floating_point() or b.is_complex()):
        b = b.float()
    return a, b


def logaddexp(x1, x2, out=None) -> DNDarray:
    return _operations.binary_op(lambda a, b: torch.logaddexp(*_floatify(a, b)), x1, x2, out)


def logaddexp2(x1, x2, out=None) -> DNDarray:
    return _operations.binary_op(lambda a, b: torch.logaddexp2(*_floatify(a, b)), x1, x2, out)


def sqrt(x, out=None) -> DNDarray:
    return _operations.local_op(torch.sqrt, x, out)


def square(x, out=None) -> DNDarray:
    return _operations.local_op(torch.square, x, out)


for _n in ("exp", "expm1", "exp2", "log", "log2", "log10", "log1p", "sqrt", "square"):
    setattr(DNDarray, _n, (lambda f: lambda self, out=None: f(self, out))(globals()[_n]))
