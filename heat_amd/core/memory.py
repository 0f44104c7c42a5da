"""Memory-layout helpers (reference ``heat/core/memory.py``: ``copy`` 13, ``sanitize_memory_layout`` 42)."""
from __future__ import annotations

import torch

from . import sanitation
from .dndarray import DNDarray

__all__ = ["copy", "sanitize_memory_layout"]


def copy(x: DNDarray) -> DNDarray:
    """Deep copy of a DNDarray (same split/balance metadata, no communication)."""
    sanitation.sanitize_in(x)
    return DNDarray(x.larray.clone(), x.shape, x.dtype, x.split, x.device, x.comm, x.balanced)


DNDarray.copy = lambda self: copy(self)
DNDarray.copy.__doc__ = copy.__doc__


def sanitize_memory_layout(x: torch.Tensor, order: str = "C") -> torch.Tensor:
    """Return ``x`` laid out row-major ('C') or column-major ('F'), values unchanged."""
    if order == "K":
        raise NotImplementedError("order='K' is not supported; use 'C' (row-major) or 'F' (column-major)")
    if x.ndim < 2 or x.numel() == 0:
        return x
    strides = x.stride()
    column_major = all(strides[i] <= strides[i + 1] for i in range(x.ndim - 1))
    row_major = not column_major
    if (order == "C" and row_major) or (order == "F" and column_major):
        return x
    if order == "C":
        return x.contiguous()
    if order == "F":
        # column-major: the transposed tensor is contiguous
        return x.permute(*reversed(range(x.ndim))).contiguous().permute(*reversed(range(x.ndim)))
    raise ValueError("combination of order and layout not permitted, order: {} column major: {} row major: {}"
                     .format(order, column_major, row_major))
