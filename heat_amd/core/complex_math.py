"""Complex number helpers (reference ``heat/core/complex_math.py``)."""
from __future__ import annotations

import torch

from . import _operations, types
from .dndarray import DNDarray

__all__ = ["angle", "conj", "conjugate", "imag", "real"]


def angle(x, deg: bool = False, out=None) -> DNDarray:
    """Argument of complex numbers (radians, or degrees with ``deg``)."""
    res = _operations.local_op(torch.angle, x, out)
    if deg:
        res *= 180.0 / 3.141592653589793
    return res


def conjugate(x, out=None) -> DNDarray:
    """Element-wise complex conjugate (a copy for real input). Local op, split preserved."""
    return _operations.local_op(lambda t: torch.conj(t).resolve_conj(), x, out, no_cast=True)


conj = conjugate


def imag(x) -> DNDarray:
    """Imaginary part (zeros of the same shape for real input). Local op, split preserved."""
    if types.heat_type_is_complexfloating(x.dtype):
        return _operations.local_op(lambda t: torch.imag(t).clone(), x, no_cast=True)
    from . import factories

    return factories.zeros_like(x)


def real(x) -> DNDarray:
    """Real part (the array itself for real input). Local op, split preserved."""
    if types.heat_type_is_complexfloating(x.dtype):
        return _operations.local_op(lambda t: torch.real(t).clone(), x, no_cast=True)
    return x


DNDarray.conj = lambda self, out=None: conjugate(self, out)
DNDarray.angle = lambda self, deg=False, out=None: angle(self, deg, out)
