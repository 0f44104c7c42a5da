"""Rounding functions (reference ``heat/core/rounding.py``)."""
from __future__ import annotations

import torch

from . import _operations, types
from .dndarray import DNDarray

__all__ = ["abs", "absolute", "ceil", "clip", "fabs", "floor", "modf", "round", "trunc"]


def abs(x, out=None, dtype=None) -> DNDarray:
    """Element-wise absolute value (optionally cast to ``dtype``)."""
    if dtype is not None and not (isinstance(dtype, type) and issubclass(dtype, types.datatype)):
        raise TypeError("dtype must be a heat data type, got {}".format(dtype))
    res = _operations.local_op(torch.abs, x, out, no_cast=True)
    if dtype is not None:
        res = res.astype(dtype, copy=False)
    return res


absolute = abs


def fabs(x, out=None) -> DNDarray:
    """Absolute value as floating point."""
    if not isinstance(x, DNDarray):
        raise TypeError("expected x to be a DNDarray, but was {}".format(type(x)))
    return abs(x, out, dtype=None if types.heat_type_is_inexact(x.dtype) else types.promote_types(x.dtype, types.float32))


def ceil(x, out=None) -> DNDarray:
    """Element-wise ceiling (smallest integer-valued float >= x). Local op, split preserved."""
    return _operations.local_op(torch.ceil, x, out)


def floor(x, out=None) -> DNDarray:
    """Element-wise floor (largest integer-valued float <= x). Local op, split preserved."""
    return _operations.local_op(torch.floor, x, out)


def trunc(x, out=None) -> DNDarray:
    """Element-wise truncation toward zero. Local op, split preserved."""
    return _operations.local_op(torch.trunc, x, out)


def round(x, decimals: int = 0, out=None, dtype=None) -> DNDarray:
    """Round half to even to the given number of decimals."""
    if dtype is not None and not (isinstance(dtype, type) and issubclass(dtype, types.datatype)):
        raise TypeError("dtype must be a heat data type, got {}".format(dtype))

    def _round(t, decimals=decimals):
        if decimals == 0:
            return torch.round(t)
        return torch.round(t, decimals=decimals)

    res = _operations.local_op(_round, x, out)
    if dtype is not None:
        res = res.astype(dtype, copy=False)
    return res


def clip(x, min=None, max=None, out=None) -> DNDarray:
    """Limit values to ``[min, max]``."""
    if not isinstance(x, DNDarray):
        raise TypeError("a must be a DNDarray, but is {}".format(type(x)))
    if min is None and max is None:
        raise ValueError("either min or max must be set")
    lo = min.larray if isinstance(min, DNDarray) else min
    hi = max.larray if isinstance(max, DNDarray) else max
    return _operations.local_op(lambda t: torch.clamp(t, lo, hi), x, out, no_cast=True)


def modf(x, out=None):
    """Fractional and integral parts, both with the sign of x."""
    if not isinstance(x, DNDarray):
        raise TypeError("expected x to be a DNDarray, but was {}".format(type(x)))
    integral = trunc(x)
    fractional = x - integral
    if out is not None:
        if not isinstance(out, tuple):
            raise TypeError("expected out to be None or a tuple of two DNDarrays, got {}".format(type(out)))
        if len(out) != 2:
            raise ValueError("expected out to be a tuple of two DNDarrays, got {} entries".format(len(out)))
        if not all(isinstance(o, DNDarray) for o in out):
            raise TypeError("expected out to hold two DNDarrays")
        out[0].larray.copy_(fractional.larray)
        out[1].larray.copy_(integral.larray)
        return out
    return fractional, integral


DNDarray.__abs__ = lambda self: abs(self)
DNDarray.abs = lambda self, out=None, dtype=None: abs(self, out, dtype)
DNDarray.absolute = DNDarray.abs
DNDarray.ceil = lambda self, out=None: ceil(self, out)
DNDarray.floor = lambda self, out=None: floor(self, out)
DNDarray.trunc = lambda self, out=None: trunc(self, out)
DNDarray.round = lambda self, decimals=0, out=None, dtype=None: round(self, decimals, out, dtype)
DNDarray.clip = lambda self, min=None, max=None, out=None: clip(self, min, max, out)
DNDarray.fabs = lambda self, out=None: fabs(self, out)
DNDarray.modf = lambda self, out=None: modf(self, out)
