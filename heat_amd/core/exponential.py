"""Exponential and logarithmic functions (reference ``heat/core/exponential.py``)."""
from __future__ import annotations

import torch

from . import _operations
from .dndarray import DNDarray

__all__ = ["exp", "expm1", "exp2", "log", "log2", "log10", "log1p", "logaddexp", "logaddexp2", "sqrt", "square"]


def exp(x, out=None) -> DNDarray:
    """Element-wise exponential e**x; integer input is promoted to float32. Split and device of ``x`` are kept
    (a local op: no communication). Reference ``heat/core/exponential.py: exp``."""
    return _operations.local_op(torch.exp, x, out)


def expm1(x, out=None) -> DNDarray:
    """Element-wise e**x - 1, accurate for small ``x``. Local op, split preserved."""
    return _operations.local_op(torch.expm1, x, out)


def exp2(x, out=None) -> DNDarray:
    """Element-wise 2**x. Local op, split preserved."""
    return _operations.local_op(torch.exp2, x, out)


def log(x, out=None) -> DNDarray:
    """Element-wise natural logarithm (nan for x < 0, -inf at 0). Local op, split preserved."""
    return _operations.local_op(torch.log, x, out)


def log2(x, out=None) -> DNDarray:
    """Element-wise base-2 logarithm. Local op, split preserved."""
    return _operations.local_op(torch.log2, x, out)


def log10(x, out=None) -> DNDarray:
    """Element-wise base-10 logarithm. Local op, split preserved."""
    return _operations.local_op(torch.log10, x, out)


def log1p(x, out=None) -> DNDarray:
    """Element-wise log(1 + x), accurate for small ``x``. Local op, split preserved."""
    return _operations.local_op(torch.log1p, x, out)


def _floatify(a, b):
    if not (a.is_floating_point() or a.is_complex()):
        a = a.float()
    if not (b.is_floating_point() or b.is_complex()):
        b = b.float()
    return a, b


def logaddexp(x1, x2, out=None) -> DNDarray:
    """log(exp(x1) + exp(x2)) element-wise without overflow; operands broadcast (a split operand is
    aligned with the other by the binary-op engine), integers promote to float."""
    return _operations.binary_op(lambda a, b: torch.logaddexp(*_floatify(a, b)), x1, x2, out)


def logaddexp2(x1, x2, out=None) -> DNDarray:
    """log2(2**x1 + 2**x2) element-wise without overflow; broadcasting as ``logaddexp``."""
    return _operations.binary_op(lambda a, b: torch.logaddexp2(*_floatify(a, b)), x1, x2, out)


def sqrt(x, out=None) -> DNDarray:
    """Element-wise non-negative square root (nan for negative input). Local op, split preserved."""
    return _operations.local_op(torch.sqrt, x, out)


def square(x, out=None) -> DNDarray:
    """Element-wise x * x. Local op, split and dtype preserved."""
    return _operations.local_op(torch.square, x, out)


for _n in ("exp", "expm1", "exp2", "log", "log2", "log10", "log1p", "sqrt", "square"):
    setattr(DNDarray, _n, (lambda f: lambda self, out=None: f(self, out))(globals()[_n]))
