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

    def take_x(c, a):
        return torch.where(c.bool(), a.to(tt), torch.zeros((), dtype=tt, device=a.device))

    def take_y(c, b):
        return torch.where(c.bool(), torch.zeros((), dtype=tt, device=b.device), b.to(tt))

    # the two halves are disjoint, so their sum is the selection (exact: one term is always 0)
    px = _operations.binary_op(take_x, cond, x)
    py = _operations.binary_op(take_y, cond, y)
    res = _operations.binary_op(torch.add, px, py)
    return DNDarray(res.larray.to(tt), res.gshape, dtype, res.split, res.device, res.comm, res.balanced)


DNDarray.nonzero = lambda self: nonzero(self)
