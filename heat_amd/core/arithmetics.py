"""
Arithmetic operations (reference ``heat/core/arithmetics.py``: ``add`` 91 … ``sum`` 943, ``diff``
halo exchange 380-420, ``cumsum/cumprod`` 290/250).
"""
from __future__ import annotations

from typing import Optional, Tuple, Union

import torch

from . import _operations, types
from .communication import MPI
from .dndarray import DNDarray
from .stride_tricks import sanitize_axis

__all__ = ["add", "bitwise_and", "bitwise_not", "bitwise_or", "bitwise_xor", "cumprod", "cumproduct",
           "cumsum", "diff", "div", "divide", "floordiv", "floor_divide", "fmod", "invert", "left_shift",
           "mod", "mul", "multiply", "neg", "negative", "pos", "positive", "pow", "power", "prod",
           "remainder", "right_shift", "sub", "subtract", "sum"]


def _check_exact(t1, t2, name):
    for t in (t1, t2):
        ty = types.heat_type_of(t)
        if not (types.heat_type_is_exact(ty) or ty is types.bool):
            raise TypeError("Operation {} is not supported for the data type {}".format(name, ty))


def add(t1, t2, out=None, where=True) -> DNDarray:
    """Element-wise addition."""
    return _operations.binary_op(torch.add, t1, t2, out, where)


def sub(t1, t2, out=None, where=True) -> DNDarray:
    """Element-wise subtraction."""
    return _operations.binary_op(torch.sub, t1, t2, out, where)


subtract = sub


def mul(t1, t2, out=None, where=True) -> DNDarray:
    """Element-wise multiplication."""
    return _operations.binary_op(torch.mul, t1, t2, out, where)


multiply = mul


def div(t1, t2, out=None, where=True) -> DNDarray:
    """Element-wise true division (integers promote to floating point)."""
    return _operations.binary_op(torch.true_divide, t1, t2, out, where)


divide = div


def floordiv(t1, t2, out=None, where=True) -> DNDarray:
    """Element-wise floor division."""
    return _operations.binary_op(lambda a, b: torch.div(a, b, rounding_mode="floor"), t1, t2, out, where)


floor_divide = floordiv


def fmod(t1, t2, out=None, where=True) -> DNDarray:
    """Element-wise C-style remainder (sign of the dividend)."""
    return _operations.binary_op(torch.fmod, t1, t2, out, where)


def mod(t1, t2, out=None, where=True) -> DNDarray:
    """Element-wise Python-style remainder (sign of the divisor)."""
    return _operations.binary_op(torch.remainder, t1, t2, out, where)


remainder = mod


def pow(t1, t2, out=None, where=True) -> DNDarray:
    """Element-wise power."""
    return _operations.binary_op(torch.pow, t1, t2, out, where)


power = pow


def bitwise_and(t1, t2, out=None, where=True) -> DNDarray:
    """Element-wise bitwise AND of integer or boolean operands (floats raise TypeError); ``where``
    masks the positions written."""
    _check_exact(t1, t2, "bitwise_and")
    return _operations.binary_op(torch.bitwise_and, t1, t2, out, where)


def bitwise_or(t1, t2, out=None, where=True) -> DNDarray:
    """Element-wise bitwise OR of integer or boolean operands (floats raise TypeError)."""
    _check_exact(t1, t2, "bitwise_or")
    return _operations.binary_op(torch.bitwise_or, t1, t2, out, where)


def bitwise_xor(t1, t2, out=None, where=True) -> DNDarray:
    """Element-wise bitwise XOR of integer or boolean operands (floats raise TypeError)."""
    _check_exact(t1, t2, "bitwise_xor")
    return _operations.binary_op(torch.bitwise_xor, t1, t2, out, where)


def invert(a, out=None) -> DNDarray:
    """Bitwise NOT (logical NOT for booleans)."""
    if not (types.heat_type_is_exact(a.dtype) or a.dtype is types.bool):
        raise TypeError("Operation is not supported for the data type {}".format(a.dtype))
    return _operations.local_op(torch.bitwise_not, a, out, no_cast=True)


bitwise_not = invert


def left_shift(t1, t2, out=None, where=True) -> DNDarray:
    """Element-wise ``t1 << t2`` for integer operands (floats raise TypeError)."""
    _check_exact(t1, t2, "left_shift")
    return _operations.binary_op(torch.bitwise_left_shift, t1, t2, out, where)


def right_shift(t1, t2, out=None, where=True) -> DNDarray:
    """Element-wise ``t1 >> t2`` (arithmetic shift) for integer operands (floats raise TypeError)."""
    _check_exact(t1, t2, "right_shift")
    return _operations.binary_op(torch.bitwise_right_shift, t1, t2, out, where)


def neg(a, out=None) -> DNDarray:
    """Element-wise negation."""
    return _operations.local_op(torch.neg, a, out, no_cast=True)


negative = neg


def pos(a, out=None) -> DNDarray:
    """Element-wise unary plus (a copy)."""
    def positive_fn(t, out=None):
        return t.clone()

    return _operations.local_op(positive_fn, a, out, no_cast=True)


positive = pos


def _cum_dtype(a, dtype):
    if dtype is not None:
        return dtype
    if a.dtype is types.bool:
        return types.int64
    return None


def cumsum(a, axis: int, dtype=None, out=None) -> DNDarray:
    """Cumulative sum along ``axis`` (carry across ranks by one all-gather)."""
    return _operations.cum_op(a, torch.cumsum, MPI.SUM, torch.add, 0, axis, _cum_dtype(a, dtype), out)


def cumprod(a, axis: int, dtype=None, out=None) -> DNDarray:
    """Cumulative product along ``axis``."""
    return _operations.cum_op(a, torch.cumprod, MPI.PROD, torch.mul, 1, axis, _cum_dtype(a, dtype), out)


cumproduct = cumprod


def diff(a, n: int = 1, axis: int = -1, prepend=None, append=None) -> DNDarray:
    """n-th discrete difference along ``axis``; along the split axis one halo slice is exchanged."""
    from . import factories, manipulations

    if n == 0:
        return a
    if n < 0:
        raise ValueError("diff requires that n be a positive number, got {}".format(n))
    if not isinstance(a, DNDarray):
        raise TypeError("'a' must be a DNDarray")
    axis = sanitize_axis(a.gshape, axis)
    if prepend is not None or append is not None:
        parts = []
        for extra in (prepend,):
            if extra is not None:
                parts.append(_as_edge(extra, a, axis))
        parts.append(a)
        if append is not None:
            parts.append(_as_edge(append, a, axis))
        a = manipulations.concatenate(parts, axis=axis)
    if not a.is_distributed() or axis != a.split:
        res = torch.diff(a.larray, n=n, dim=axis)
        gshape = list(a.gshape)
        gshape[axis] = max(0, gshape[axis] - n)
        return DNDarray(res, tuple(gshape), types.canonical_heat_type(res.dtype), a.split, a.device, a.comm,
                        a.balanced)
    out = a
    for _ in range(n):
        out = _diff_once_split(out, axis)
    return out


def _as_edge(v, a, axis):
    from . import factories

    if isinstance(v, DNDarray):
        return v
    shape = list(a.gshape)
    shape[axis] = 1
    t = torch.as_tensor(v, dtype=a.larray.dtype, device=a.larray.device)
    t = t.expand(shape).contiguous() if t.dim() == 0 or t.numel() == 1 else t.reshape(shape)
    return factories.array(t, device=a.device, comm=a.comm)


def _diff_once_split(a: DNDarray, axis: int) -> DNDarray:
    a.get_halo(1)
    t = a.larray
    nxt = a.halo_next
    ext = torch.cat([t, nxt], dim=axis) if nxt is not None else t
    res = torch.diff(ext, n=1, dim=axis)
    gshape = list(a.gshape)
    gshape[axis] -= 1
    out = DNDarray(res, tuple(gshape), types.canonical_heat_type(res.dtype), a.split, a.device, a.comm, None)
    return out


def prod(a, axis=None, out=None, keepdim=False) -> DNDarray:
    """Product of elements over the given axis / axes."""
    def _prod(t, dim, keepdim):
        return torch.prod(t, dim=dim, keepdim=keepdim)

    return _operations.reduce_op(a, _prod, MPI.PROD, axis=axis, out=out, neutral=1, keepdim=keepdim)


def sum(a, axis=None, out=None, keepdim=False) -> DNDarray:
    """Sum of elements over the given axis / axes."""
    def _sum(t, dim, keepdim):
        return torch.sum(t, dim=dim, keepdim=keepdim)

    return _operations.reduce_op(a, _sum, MPI.SUM, axis=axis, out=out, neutral=0, keepdim=keepdim)


# ---------------------------------------------------------------------------------------------
# DNDarray operator overloads
# ---------------------------------------------------------------------------------------------
def _r(fn):
    return lambda self, other: fn(other, self)


DNDarray.__add__ = lambda self, other: add(self, other)
DNDarray.__radd__ = _r(add)
DNDarray.__sub__ = lambda self, other: sub(self, other)
DNDarray.__rsub__ = _r(sub)
DNDarray.__mul__ = lambda self, other: mul(self, other)
DNDarray.__rmul__ = _r(mul)
DNDarray.__truediv__ = lambda self, other: div(self, other)
DNDarray.__rtruediv__ = _r(div)
DNDarray.__floordiv__ = lambda self, other: floordiv(self, other)
DNDarray.__rfloordiv__ = _r(floordiv)
DNDarray.__mod__ = lambda self, other: mod(self, other)
DNDarray.__rmod__ = _r(mod)
DNDarray.__pow__ = lambda self, other: pow(self, other)
DNDarray.__rpow__ = _r(pow)
DNDarray.__and__ = lambda self, other: bitwise_and(self, other)
DNDarray.__rand__ = _r(bitwise_and)
DNDarray.__or__ = lambda self, other: bitwise_or(self, other)
DNDarray.__ror__ = _r(bitwise_or)
DNDarray.__xor__ = lambda self, other: bitwise_xor(self, other)
DNDarray.__rxor__ = _r(bitwise_xor)
DNDarray.__invert__ = lambda self: invert(self)
DNDarray.__lshift__ = lambda self, other: left_shift(self, other)
DNDarray.__rlshift__ = _r(left_shift)
DNDarray.__rshift__ = lambda self, other: right_shift(self, other)
DNDarray.__rrshift__ = _r(right_shift)
DNDarray.__neg__ = lambda self: neg(self)
DNDarray.__pos__ = lambda self: pos(self)
DNDarray.prod = lambda self, axis=None, out=None, keepdim=False: prod(self, axis, out, keepdim)
DNDarray.sum = lambda self, axis=None, out=None, keepdim=False: sum(self, axis, out, keepdim)
DNDarray.cumsum = lambda self, axis, dtype=None, out=None: cumsum(self, axis, dtype, out)
DNDarray.cumprod = lambda self, axis, dtype=None, out=None: cumprod(self, axis, dtype, out)
