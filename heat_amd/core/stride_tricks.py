"""Shape and axis helpers (reference ``heat/core/stride_tricks.py``: ``broadcast_shape`` 11,
``sanitize_axis`` 57, ``sanitize_shape`` 120, ``sanitize_slice`` 165)."""
from __future__ import annotations

from typing import Tuple, Union

import numpy as np

__all__ = ["broadcast_shape", "broadcast_shapes", "sanitize_axis", "sanitize_shape", "sanitize_slice"]


def broadcast_shape(shape_a: Tuple[int, ...], shape_b: Tuple[int, ...]) -> Tuple[int, ...]:
    """NumPy broadcasting of two shapes; raises ValueError if incompatible."""
    la, lb = len(shape_a), len(shape_b)
    n = max(la, lb)
    out = []
    for i in range(1, n + 1):
        a = shape_a[-i] if i <= la else 1
        b = shape_b[-i] if i <= lb else 1
        if a != b and a != 1 and b != 1:
            raise ValueError("operands could not be broadcast, input shapes {} {}".format(shape_a, shape_b))
        out.append(b if a == 1 else a)
    return tuple(reversed(out))


def broadcast_shapes(*shapes) -> Tuple[int, ...]:
    res = ()
    for s in shapes:
        res = broadcast_shape(res, tuple(s))
    return res


def sanitize_axis(shape: Tuple[int, ...], axis) -> Union[int, None, Tuple[int, ...]]:
    """Normalise a (possibly negative) axis or tuple of axes against ``shape``."""
    if len(shape) == 0:
        axis = None
    if axis is None:
        return None
    if isinstance(axis, (np.integer,)):
        axis = int(axis)
    if isinstance(axis, list):
        axis = tuple(axis)
    if isinstance(axis, bool) or not isinstance(axis, (int, tuple)):
        raise TypeError("axis must be None or int or tuple, but was {}".format(type(axis)))
    nd = len(shape)
    if isinstance(axis, tuple):
        res = []
        for a in axis:
            if not isinstance(a, (int, np.integer)):
                raise TypeError("axis must be None or int or tuple, but was {}".format(type(a)))
            a = int(a) + nd if a < 0 else int(a)
            if a < 0 or a >= nd:
                raise ValueError("axis {} is out of bounds for shape {}".format(axis, shape))
            res.append(a)
        return tuple(res)
    a = axis + nd if axis < 0 else axis
    if a < 0 or a >= nd:
        raise ValueError("axis {} is out of bounds for shape {}".format(axis, shape))
    return a


def sanitize_shape(shape, lval: int = 0) -> Tuple[int, ...]:
    """Normalise an int or sequence of ints into a shape tuple."""
    shape = tuple(shape) if hasattr(shape, "__iter__") else (shape,)
    out = []
    for d in shape:
        if isinstance(d, np.integer):
            d = int(d)
        if hasattr(d, "item") and not isinstance(d, int):
            try:
                d = d.item()
            except Exception:
                pass
        if isinstance(d, bool) or not isinstance(d, int):
            raise TypeError("expected sequence object with length >= 0 or a single integer")
        if d < lval:
            raise ValueError("negative dimensions are not allowed")
        out.append(d)
    return tuple(out)


def sanitize_slice(sl: slice, max_dim: int) -> slice:
    """Replace None members of a slice and resolve negative bounds."""
    if not isinstance(sl, slice):
        raise TypeError("This function is only for slices!")
    start = 0 if sl.start is None else sl.start
    if start < 0:
        start += max_dim
    stop = max_dim if sl.stop is None else sl.stop
    if stop < 0:
        stop += max_dim
    step = 1 if sl.step is None else sl.step
    return slice(start, stop, step)
