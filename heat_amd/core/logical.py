"""Logical functions (reference ``heat/core/logical.py``: ``all`` 37, ``allclose`` 104 (Allreduce LAND
144), ``any`` 157, ``isclose`` 204, ``isfinite/isinf/isnan`` …, ``logical_*``, ``signbit``)."""
from __future__ import annotations

from typing import Optional

import numpy as np
import torch

from . import _operations, types
from .communication import MPI
from .dndarray import DNDarray

__all__ = ["all", "allclose", "any", "isclose", "isfinite", "isinf", "isnan", "isneginf", "isposinf",
           "logical_and", "logical_not", "logical_or", "logical_xor", "signbit"]


def all(x, axis=None, out=None, keepdim: bool = False) -> DNDarray:
    """Whether all elements (along ``axis``) evaluate to True."""
    def _all(t, dim, keepdim):
        return torch.all(t.bool(), dim=dim, keepdim=keepdim)

    return _operations.reduce_op(x, _all, MPI.LAND, axis=axis, out=out, neutral=1, keepdim=keepdim)


def any(x, axis=None, out=None, keepdim: bool = False) -> DNDarray:
    """Whether any element (along ``axis``) evaluates to True."""
    def _any(t, dim, keepdim):
        return torch.any(t.bool(), dim=dim, keepdim=keepdim)

    return _operations.reduce_op(x, _any, MPI.LOR, axis=axis, out=out, neutral=0, keepdim=keepdim)


def _as_array(v, like: DNDarray):
    from . import factories

    if isinstance(v, DNDarray):
        return v
    return factories.array(v, device=like.device, comm=like.comm)


def isclose(x, y, rtol: float = 1e-05, atol: float = 1e-08, equal_nan: bool = False) -> DNDarray:
    """Element-wise closeness test ``|x - y| <= atol + rtol * |y|``."""
    def _isclose(a, b):
        if a.dtype != b.dtype:
            common = torch.promote_types(a.dtype, b.dtype)
            if not (common.is_floating_point or common.is_complex):
                common = torch.float32
            a, b = a.to(common), b.to(common)
        return torch.isclose(a, b, rtol=rtol, atol=atol, equal_nan=equal_nan)

    for v in (x, y):
        if not isinstance(v, (DNDarray, int, float, bool, np.number)):
            raise TypeError("Only DNDarrays and numeric scalars are supported, got {}".format(type(v)))
    if not isinstance(x, DNDarray) and not isinstance(y, DNDarray):
        # two scalars: a plain bool like the reference
        return bool(abs(x - y) <= atol + rtol * abs(y) or (equal_nan and x != x and y != y))
    return _operations.binary_op(_isclose, x, y)


def allclose(x, y, rtol: float = 1e-05, atol: float = 1e-08, equal_nan: bool = False) -> bool:
    """True when every element pair is close (one all-reduce of a boolean)."""
    for v in (x, y):
        if not isinstance(v, (DNDarray, int, float, bool, np.number)):
            raise TypeError("Only DNDarrays and numeric scalars are supported, got {}".format(type(v)))
    if not isinstance(x, DNDarray):
        x = _as_array(x, y)
    if not isinstance(y, DNDarray):
        y = _as_array(y, x)
    close = isclose(x, y, rtol, atol, equal_nan)
    ok = torch.tensor([bool(torch.all(close.larray))], dtype=torch.uint8, device=close.larray.device)
    if close.is_distributed():
        close.comm.Allreduce(MPI.IN_PLACE, ok, MPI.LAND)
    return bool(ok.item())


def isfinite(x) -> DNDarray:
    """Element-wise test for finite values (not inf, not nan); boolean result, split preserved."""
    return _operations.local_op(torch.isfinite, x, no_cast=True)


def isinf(x) -> DNDarray:
    """Element-wise test for +inf or -inf; boolean result, split preserved."""
    return _operations.local_op(torch.isinf, x, no_cast=True)


def isnan(x) -> DNDarray:
    """Element-wise test for nan; boolean result, split preserved."""
    return _operations.local_op(torch.isnan, x, no_cast=True)


def isneginf(x, out=None) -> DNDarray:
    """Element-wise test for -inf; boolean result, split preserved."""
    return _operations.local_op(torch.isneginf, x, out, no_cast=True)


def isposinf(x, out=None) -> DNDarray:
    """Element-wise test for +inf; boolean result, split preserved."""
    return _operations.local_op(torch.isposinf, x, out, no_cast=True)


def logical_and(t1, t2) -> DNDarray:
    """Element-wise truth-value AND of two operands (non-zero is True); broadcasting binary op."""
    return _operations.binary_op(lambda a, b: torch.logical_and(a.bool(), b.bool()), t1, t2)


def logical_or(t1, t2) -> DNDarray:
    """Element-wise truth-value OR of two operands (non-zero is True); broadcasting binary op."""
    return _operations.binary_op(lambda a, b: torch.logical_or(a.bool(), b.bool()), t1, t2)


def logical_xor(t1, t2) -> DNDarray:
    """Element-wise truth-value XOR of two operands (non-zero is True); broadcasting binary op."""
    return _operations.binary_op(lambda a, b: torch.logical_xor(a.bool(), b.bool()), t1, t2)


def logical_not(t, out=None) -> DNDarray:
    """Element-wise truth-value NOT; boolean result, split preserved."""
    return _operations.local_op(torch.logical_not, t, out, no_cast=True)


def signbit(x, out=None) -> DNDarray:
    """True where the sign bit is set (negative numbers, -0.0)."""
    return _operations.local_op(torch.signbit, x, out, no_cast=True)


DNDarray.all = lambda self, axis=None, out=None, keepdim=False: all(self, axis, out, keepdim)
DNDarray.any = lambda self, axis=None, out=None, keepdim=False: any(self, axis, out, keepdim)
DNDarray.allclose = lambda self, other, rtol=1e-05, atol=1e-08, equal_nan=False: allclose(self, other, rtol, atol, equal_nan)
DNDarray.isclose = lambda self, other, rtol=1e-05, atol=1e-08, equal_nan=False: isclose(self, other, rtol, atol, equal_nan)
