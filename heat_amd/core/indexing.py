"""Index-returning functions (reference ``heat/core/indexing.py``: ``nonzero`` 16, ``where`` 93)."""
from __future__ import annotations

from typing import Union

import torch

from . import _operations, types
from .communication import MPI
from .dndarray import DNDarray

__all__ = ["nonzero", "where"]


def nonzero(x: DNDarray) -> DNDarray:
    """Global coordinates of the non-zero elements, one row per element (split 0, unbalanced,
    when ``x`` is split; a 1-D input gives a 1-D result). ``x[nonzero(x)]`` selects them."""
    if not isinstance(x, DNDarray):
        raise TypeError("Input must be a DNDarray, is {}".format(type(x)))
    t = x.larray
    nz = torch.nonzero(t, as_tuple=False)
    balanced = None
    if x.is_distributed():
        counts, displs = x.counts_displs()
        nz[:, x.split] += displs[x.comm.rank]
        if x.split == 0:
            # rank blocks are already in C order: keep the local rows (unbalanced, no traffic)
            total = x.comm.allreduce(int(nz.shape[0]), MPI.SUM)
        else:
            # split > 0: rank order is not C order - place every row at its global C position
            # (per-outer-index counts + one exchange; the reference returns rank order here)
            pos, total = x._mask_positions(t != 0)
            nz = x._place_by_position(nz, pos, total)
            balanced = True
        split = 0
    else:
        total = int(nz.shape[0])
        split = None if x.split is None else 0
    if x.ndim == 1:
        nz = nz.squeeze(1)
        gshape = (total,)
    else:
        gshape = (total, x.ndim)
    return DNDarray(nz, gshape, types.int64, split, x.device, x.comm,
                    balanced if split is not None else True)


def where(cond: DNDarray, x=None, y=None) -> DNDarray:
    """Elements of ``x`` where ``cond`` holds, else of ``y``; with only ``cond``: :func:`nonzero`."""
    if x is None and y is None:
        return nonzero(cond)
    if x is None or y is None:
        raise TypeError("either both or neither x and y must be given")
    if not isinstance(cond, DNDarray):
        raise TypeError("cond must be a DNDarray")
    for v in (x, y):
        if not isinstance(v, (DNDarray, int, float, bool)):
            raise TypeError("x and y must be DNDarrays or numerical scalars, got {}".format(type(v)))

    dtype = types.result_type(x, y)
    tt = dtype.torch_type()

    # identically distributed operands (the common case, e.g. a mask computed from x): ONE
    # torch.where on the local blocks - the generic path below makes three passes
    arrs = [v for v in (cond, x, y) if isinstance(v, DNDarray)]
    dev = cond.larray.device
    if all(v.gshape == cond.gshape and v.split == cond.split and v.larray.device == dev for v in arrs) and \
            (not cond.is_distributed() or all(v.balanced for v in arrs)):
        xa = x.larray.to(tt) if isinstance(x, DNDarray) else torch.tensor(x, dtype=tt, device=dev)
        ya = y.larray.to(tt) if isinstance(y, DNDarray) else torch.tensor(y, dtype=tt, device=dev)
        res = torch.where(cond.larray.bool(), xa, ya)
        if res.shape != cond.larray.shape:   # 0-d operands only: broadcast to the block
            res = res.expand(cond.larray.shape).contiguous()
        return DNDarray(res, cond.gshape, dtype, cond.split, cond.device, cond.comm, cond.balanced)

    def take_x(c, a):
        return torch.where(c.bool(), a.to(tt), torch.zeros((), dtype=tt, device=a.device))

    def take_y(c, b):
        return torch.where(c.bool(), torch.zeros((), dtype=tt, device=b.device), b.to(tt))

    # the two halves are disjoint (one is all-zero bits at every position), so their bitwise OR is
    # the selection - exact for every value, -0.0 and NaN payloads included (a sum turned -0.0 into
    # +0.0)
    ibits = {1: torch.uint8, 2: torch.int16, 4: torch.int32, 8: torch.int64, 16: torch.int64}

    def merge(a, b):
        if a.dtype == torch.bool:
            return a | b
        av, bv = (torch.view_as_real(a), torch.view_as_real(b)) if a.is_complex() else (a, b)
        it = ibits[av.element_size()]
        out = (av.contiguous().view(it) | bv.contiguous().view(it)).view(av.dtype)
        return torch.view_as_complex(out) if a.is_complex() else out

    px = _operations.binary_op(take_x, cond, x)
    py = _operations.binary_op(take_y, cond, y)
    res = _operations.binary_op(merge, px, py)
    return DNDarray(res.larray.to(tt), res.gshape, dtype, res.split, res.device, res.comm, res.balanced)


DNDarray.nonzero = lambda self: nonzero(self)
