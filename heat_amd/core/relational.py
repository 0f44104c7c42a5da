"""Relational operators (reference ``heat/core/relational.py``; ``equal`` all-reduces one bool)."""
from __future__ import annotations

import torch

from . import _operations
from .communication import MPI
from .dndarray import DNDarray

__all__ = ["eq", "equal", "ge", "greater", "greater_equal", "gt", "le", "less", "less_equal", "lt", "ne",
           "not_equal"]


def eq(x, y) -> DNDarray:
    """Element-wise ``x == y`` (boolean); operands broadcast, a scalar operand is allowed."""
    return _operations.binary_op(torch.eq, x, y)


def ne(x, y) -> DNDarray:
    """Element-wise ``x != y`` (boolean); operands broadcast, a scalar operand is allowed."""
    return _operations.binary_op(torch.ne, x, y)


def ge(x, y) -> DNDarray:
    """Element-wise ``x >= y`` (boolean); operands broadcast, a scalar operand is allowed."""
    return _operations.binary_op(torch.ge, x, y)


def gt(x, y) -> DNDarray:
    """Element-wise ``x > y`` (boolean); operands broadcast, a scalar operand is allowed."""
    return _operations.binary_op(torch.gt, x, y)


def le(x, y) -> DNDarray:
    """Element-wise ``x <= y`` (boolean); operands broadcast, a scalar operand is allowed."""
    return _operations.binary_op(torch.le, x, y)


def lt(x, y) -> DNDarray:
    """Element-wise ``x < y`` (boolean); operands broadcast, a scalar operand is allowed."""
    return _operations.binary_op(torch.lt, x, y)


greater, greater_equal, less, less_equal, not_equal = gt, ge, lt, le, ne


def equal(x, y) -> bool:
    """True if both operands have the same shape and elements (global, one all-reduce)."""
    from .stride_tricks import broadcast_shape

    if isinstance(x, DNDarray) and isinstance(y, DNDarray):
        try:
            broadcast_shape(x.gshape, y.gshape)
        except ValueError:
            return False
    res = eq(x, y)
    ok = torch.tensor([bool(torch.all(res.larray))], dtype=torch.uint8, device=res.larray.device)
    if res.is_distributed():
        res.comm.Allreduce(MPI.IN_PLACE, ok, MPI.LAND)
    return bool(ok.item())


DNDarray.__eq__ = lambda self, other: eq(self, other)
DNDarray.__ne__ = lambda self, other: ne(self, other)
DNDarray.__ge__ = lambda self, other: ge(self, other)
DNDarray.__gt__ = lambda self, other: gt(self, other)
DNDarray.__le__ = lambda self, other: le(self, other)
DNDarray.__lt__ = lambda self, other: lt(self, other)
DNDarray.__hash__ = None
