"""
Array manipulation and redistribution (reference ``heat/core/manipulations.py``: ``balance`` 63,
``concatenate`` 188, ``diag`` 512, ``diagonal`` 587, ``flip`` 826, ``pad`` 1126, ``reshape`` 1815,
``roll`` 1980, ``sort`` 2258, ``split`` 2512, ``squeeze`` 2758, ``stack`` 2861, ``unique`` 3077,
``resplit`` 3351, ``tile`` 3600, ``topk`` 3856).

Every data movement along the split axis is ONE personalised exchange built by
:func:`_segment_exchange` from "which global rows does each rank hold" -> "which rows must each rank
hold": flip, roll, concatenate, pad, tile, balance and the sort rebalance all reduce to it. This
replaces the reference's per-slice (``roll`` 2057-2078), per-column (``sort`` 2394-2489) and
neighbour-chain (``concatenate`` 377-443) message patterns.
"""
from __future__ import annotations

from typing import Iterable, List, Optional, Sequence, Tuple, Union

import numpy as np
import torch

from . import factories, types
from . import _sample_sort
from .. import ops
from .communication import MPI
from .dndarray import DNDarray, _chunk_counts, _partition_bounds
from .stride_tricks import broadcast_shape, sanitize_axis, sanitize_shape

__all__ = ["balance", "column_stack", "concatenate", "diag", "diagonal", "dsplit", "expand_dims", "flatten",
           "flip", "fliplr", "flipud", "hsplit", "hstack", "moveaxis", "pad", "ravel", "redistribute",
           "repeat", "reshape", "resplit", "roll", "rot90", "row_stack", "shape", "sort", "split", "squeeze",
           "stack", "swapaxes", "tile", "topk", "unique", "vsplit", "vstack"]


# ---------------------------------------------------------------------------------------------
# the redistribution primitive
# ---------------------------------------------------------------------------------------------
def _segment_exchange(local: torch.Tensor, axis: int, comm, segs_per_rank: List[List[Tuple[int, int, int]]],
                      dst_counts: List[int]) -> torch.Tensor:
    """Generic redistribution along ``axis``.

    ``segs_per_rank[r]`` lists ``(global_start, local_start, length)`` segments: rank r's local
    rows ``[local_start, local_start+length)`` are global rows ``[global_start, ...)``. Every rank
    knows every rank's segments (they follow from metadata). The result holds global rows
    ``[t_me, t_me + dst_counts[me])`` in order. One ``all_to_all_single``.
    """
    p, me = comm.size, comm.rank
    dst = _partition_bounds(dst_counts)
    base_shape = list(local.shape)

    def pieces(r: int, q: int):
        out = []
        t0, t1 = dst[q]
        for g, l, n in segs_per_rank[r]:
            lo, hi = max(g, t0), min(g + n, t1)
            if hi > lo:
                out.append((lo, l + (lo - g), hi - lo))
        out.sort()
        return out

    if p == 1:
        ps = pieces(0, 0)
        parts = [local.narrow(axis, l, n) for _, l, n in ps]
        if not parts:
            sh = list(base_shape)
            sh[axis] = 0
            return local.new_empty(sh)
        return torch.cat(parts, dim=axis)
    blocks = []
    for q in range(p):
        ps = pieces(me, q)
        if ps:
            blocks.append(torch.cat([local.narrow(axis, l, n) for _, l, n in ps], dim=axis))
        else:
            sh = list(base_shape)
            sh[axis] = 0
            blocks.append(local.new_empty(sh))
    shapes, recv_pieces = [], []
    for r in range(p):
        ps = pieces(r, me)
        recv_pieces.append(ps)
        sh = list(base_shape)
        sh[axis] = sum(n for _, _, n in ps)
        shapes.append(tuple(sh))
    parts = comm.exchange(blocks, shapes)
    sh = list(base_shape)
    sh[axis] = dst_counts[me]
    out = local.new_empty(sh)
    t0 = dst[me][0]
    for r in range(p):
        off = 0
        for g, _, n in recv_pieces[r]:
            out.narrow(axis, g - t0, n).copy_(parts[r].narrow(axis, off, n))
            off += n
    return out


def _local_segments(x: DNDarray) -> List[List[Tuple[int, int, int]]]:
    """Segments of a (possibly unbalanced) split array in its own coordinates."""
    counts = x.split_counts()
    bounds = _partition_bounds(counts)
    return [[(s, 0, e - s)] if e > s else [] for s, e in bounds]


def _wrap(x: DNDarray, t: torch.Tensor, gshape, split, balanced=True) -> DNDarray:
    return DNDarray(t, tuple(gshape), types.canonical_heat_type(t.dtype), split, x.device, x.comm, balanced)


# ---------------------------------------------------------------------------------------------
# distribution management
# ---------------------------------------------------------------------------------------------
def balance(array: DNDarray, copy: bool = False) -> DNDarray:
    """Balance the split axis (in place unless ``copy``)."""
    cpy = array.copy() if copy else array
    cpy.balance_()
    return cpy


def redistribute(arr: DNDarray, lshape_map: torch.Tensor = None, target_map: torch.Tensor = None) -> DNDarray:
    """Copy of ``arr`` redistributed to ``target_map``."""
    arr2 = arr.copy()
    arr2.redistribute_(lshape_map=lshape_map, target_map=target_map)
    return arr2


def resplit(arr: DNDarray, axis: Optional[int] = None) -> DNDarray:
    """Copy of ``arr`` split along ``axis`` (None = replicated)."""
    axis = sanitize_axis(arr.shape, axis)
    if axis == arr.split:
        return arr.copy()
    if not arr.is_distributed() and arr.split is None and axis is not None:
        _, _, sl = arr.comm.chunk(arr.gshape, axis)
        return DNDarray(arr.larray[sl].clone(), arr.gshape, arr.dtype, axis, arr.device, arr.comm, True)
    out = DNDarray(arr.larray, arr.gshape, arr.dtype, arr.split, arr.device, arr.comm, arr.balanced)
    out.resplit_(axis)
    if out.larray.data_ptr() == arr.larray.data_ptr():
        out._set_array(out.larray.clone())
    return out


def shape(a: DNDarray) -> Tuple[int, ...]:
    """Global shape."""
    if not isinstance(a, DNDarray):
        raise TypeError("Expected a to be a DNDarray but was {}".format(type(a)))
    return a.gshape


# ---------------------------------------------------------------------------------------------
# joining
# ---------------------------------------------------------------------------------------------
def concatenate(arrays: Sequence[DNDarray], axis: int = 0) -> DNDarray:
    """Join arrays along an existing axis (one exchange when joining along the split axis)."""
    if not isinstance(arrays, (tuple, list)) or len(arrays) == 0:
        raise TypeError("arrays must be a non-empty list or a tuple")
    arrays = list(arrays)
    for a in arrays:
        if not isinstance(a, DNDarray):
            raise TypeError("All arrays must be DNDarrays, got {}".format(type(a)))
    nd = arrays[0].ndim
    axis = sanitize_axis(arrays[0].gshape, axis)
    if len(arrays) == 1:
        return arrays[0].copy()
    for a in arrays[1:]:
        if a.ndim != nd:
            raise ValueError("DNDarrays must have the same number of dimensions")
        for i in range(nd):
            if i != axis and a.gshape[i] != arrays[0].gshape[i]:
                raise ValueError("Arrays cannot be concatenated, shapes must be the same in every axis except "
                                 "the selected axis: {}, {}".format(arrays[0].gshape, a.gshape))
    splits = set(a.split for a in arrays if a.split is not None)
    if len(splits) > 1:
        raise RuntimeError("DNDarrays given have differing split axes, arr0 {} arr1 {}".format(
            arrays[0].split, [a.split for a in arrays]))
    dtype = arrays[0].dtype
    for a in arrays[1:]:
        dtype = types.promote_types(dtype, a.dtype)
    ttype = dtype.torch_type()
    gshape = list(arrays[0].gshape)
    gshape[axis] = sum(a.gshape[axis] for a in arrays)
    split = splits.pop() if splits else None
    ref = arrays[0]
    comm = ref.comm
    if split is None or not comm.is_distributed():
        t = torch.cat([a.larray.to(ttype) for a in arrays], dim=axis)
        return DNDarray(t, tuple(gshape), dtype, split, ref.device, comm, True)
    # bring replicated members to the split distribution (local slicing)
    arrays = [a if a.split is not None else resplit(a, split) for a in arrays]
    if axis != split:
        base = arrays[0]
        counts = base.split_counts()
        parts = []
        for a in arrays:
            t = a.larray
            if a.split_counts() != counts:
                t = a._exchange_rows(a.split_counts(), counts)
            parts.append(t.to(ttype))
        return DNDarray(torch.cat(parts, dim=axis), tuple(gshape), dtype, split, ref.device, comm, base.balanced)
    # joining along the split axis: segments of each input, placed at the input's offset
    p = comm.size
    offsets = np.cumsum([0] + [a.gshape[axis] for a in arrays[:-1]])
    all_counts = [a.split_counts() for a in arrays]
    segs = [[] for _ in range(p)]
    for r in range(p):
        lpos = 0
        for i, a in enumerate(arrays):
            g0 = int(offsets[i]) + sum(all_counts[i][:r])
            n = all_counts[i][r]
            if n > 0:
                segs[r].append((g0, lpos, n))
            lpos += n
    local = torch.cat([a.larray.to(ttype) for a in arrays], dim=axis)
    target = _chunk_counts(gshape[axis], p)
    t = _segment_exchange(local, axis, comm, segs, target)
    return DNDarray(t, tuple(gshape), dtype, split, ref.device, comm, True)


def _at_least_2d_col(a: DNDarray) -> DNDarray:
    if a.ndim == 1:
        return reshape(a, (a.gshape[0], 1), new_split=0 if a.split is not None else None)
    return a


def column_stack(arrays: Sequence[DNDarray]) -> DNDarray:
    """Stack 1-D arrays as columns; 2-D arrays are concatenated along axis 1 (reference
    manipulations.py:92). A distributed 1-D array becomes a column split like the 2-D operands:
    along axis 1 when they are split there (the reference's rule), along the rows otherwise (the
    reference raises for that mix)."""
    arrays = list(arrays)
    if any(a.ndim > 2 for a in arrays):
        raise ValueError("Arrays must be 1-D or 2-D")
    if all(a.ndim == 1 for a in arrays):
        return stack(arrays, axis=1)
    col_split = 1 if any(a.ndim == 2 and a.split == 1 for a in arrays) else 0
    out = []
    for a in arrays:
        if a.ndim == 1:
            c = _at_least_2d_col(a)
            if c.split is not None and c.split != col_split:
                c = resplit(c, col_split)
            out.append(c)
        else:
            out.append(a)
    return concatenate(out, axis=1)


def hstack(arrays: Sequence[DNDarray]) -> DNDarray:
    """Stack arrays column-wise: concatenation along axis 1, or along axis 0 when every input is 1-D
    (numpy semantics). Reference ``heat/core/manipulations.py: hstack``."""
    arrays = list(arrays)
    if all(a.ndim == 1 for a in arrays):
        return concatenate(arrays, axis=0)
    return concatenate(arrays, axis=1)


def _at_least_2d_row(a: DNDarray) -> DNDarray:
    if a.ndim == 1:
        return expand_dims(a, 0)
    return a


def vstack(arrays: Sequence[DNDarray]) -> DNDarray:
    """Stack row-wise; 1-D inputs become rows. A distributed 1-D input joins a row-split stack as
    a row split along axis 0 (reference ``row_stack``: reshape to (1, n) keeping split 0)."""
    arrays = list(arrays)
    target = next((a.split for a in arrays if a.ndim > 1 and a.split is not None), 0)
    rows = []
    for a in arrays:
        r = _at_least_2d_row(a)
        if a.ndim == 1 and a.split is not None and r.split != target:
            r = resplit(r, target)
        rows.append(r)
    return concatenate(rows, axis=0)


row_stack = vstack


def stack(arrays: Sequence[DNDarray], axis: int = 0, out: Optional[DNDarray] = None) -> DNDarray:
    """Join arrays of identical shape along a new axis."""
    if isinstance(arrays, DNDarray) or not isinstance(arrays, (list, tuple)):
        raise TypeError("stack expects a sequence (list or tuple) of DNDarrays, got {}".format(type(arrays)))
    arrays = list(arrays)
    if len(arrays) < 2:
        raise ValueError("stack expects a sequence of at least 2 DNDarrays")
    for a in arrays:
        if not isinstance(a, DNDarray):
            raise TypeError("all arrays must be DNDarrays")
    a0 = arrays[0]
    for a in arrays[1:]:
        if a.gshape != a0.gshape:
            raise ValueError("all input arrays must have the same shape, got {} and {}".format(a0.gshape, a.gshape))
        if a.split != a0.split:
            raise ValueError("all input arrays must have the same split axis, got {} and {}".format(a0.split, a.split))
    axis = sanitize_axis(tuple(a0.gshape) + (1,), axis)
    counts = a0.split_counts() if a0.is_distributed() else None
    dtype = a0.dtype
    for a in arrays[1:]:
        dtype = types.promote_types(dtype, a.dtype)
    ts = []
    for a in arrays:
        t = a.larray
        if counts is not None and a.split_counts() != counts:
            t = a._exchange_rows(a.split_counts(), counts)
        ts.append(t.to(dtype.torch_type()))
    res = torch.stack(ts, dim=axis)
    gshape = list(a0.gshape)
    gshape.insert(axis, len(arrays))
    split = None if a0.split is None else (a0.split + 1 if axis <= a0.split else a0.split)
    result = DNDarray(res, tuple(gshape), dtype, split, a0.device, a0.comm, a0.balanced)
    if out is not None:
        out.larray = res.to(out.larray.dtype)
        return out
    return result


# ---------------------------------------------------------------------------------------------
# shape changes
# ---------------------------------------------------------------------------------------------
def expand_dims(a: DNDarray, axis: int) -> DNDarray:
    """Insert an axis of length one."""
    if not isinstance(a, DNDarray):
        raise TypeError("expected ht.DNDarray, but was {}".format(type(a)))
    axis = sanitize_axis(tuple(a.gshape) + (1,), axis)
    gshape = list(a.gshape)
    gshape.insert(axis, 1)
    split = None if a.split is None else (a.split + 1 if axis <= a.split else a.split)
    return DNDarray(a.larray.unsqueeze(axis), tuple(gshape), a.dtype, split, a.device, a.comm, a.balanced)


def squeeze(x: DNDarray, axis=None) -> DNDarray:
    """Remove axes of length one (a squeezed split axis becomes replicated)."""
    if not isinstance(x, DNDarray):
        raise TypeError("expected x to be a DNDarray, but was {}".format(type(x)))
    axis = sanitize_axis(x.gshape, axis)
    if axis is None:
        axes = tuple(i for i, s in enumerate(x.gshape) if s == 1)
    else:
        axes = (axis,) if isinstance(axis, int) else axis
        for a in axes:
            if x.gshape[a] != 1:
                raise ValueError("Dimension along axis {} is not 1 for shape {}".format(a, x.gshape))
    if len(axes) == 0:
        return x.copy() if False else x
    src = x
    if x.split is not None and x.split in axes and x.is_distributed():
        src = resplit(x, None)
    t = src.larray
    for a in sorted(axes, reverse=True):
        t = t.squeeze(a)
    gshape = tuple(s for i, s in enumerate(x.gshape) if i not in axes)
    if src.split is None:
        split = None
    else:
        split = src.split - sum(1 for a in axes if a < src.split)
    return DNDarray(t, gshape, x.dtype, split, x.device, x.comm, src.balanced if split is not None else True)


def reshape(a: DNDarray, *shape, **kwargs) -> DNDarray:
    """Give a new shape without changing the data (``new_split=`` selects the result split).

    Distributed: the C-order flat index of a split-0 array is contiguous per rank, so the data moves
    as flat segments in one exchange (split != 0 is first brought to split 0)."""
    if not isinstance(a, DNDarray):
        raise TypeError("'a' must be a DNDarray, currently {}".format(type(a)))
    if len(shape) == 1 and isinstance(shape[0], (list, tuple)):
        shape = tuple(shape[0])
    shape = list(shape)
    if shape.count(-1) > 1:
        raise ValueError("too many unknown dimensions")
    n = a.gnumel
    if -1 in shape:
        known = int(np.prod([s for s in shape if s != -1])) if len(shape) > 1 else 1
        if known == 0 or n % known:
            raise ValueError("cannot reshape array of size {} into shape {}".format(n, tuple(shape)))
        shape[shape.index(-1)] = n // known
    shape = sanitize_shape(shape)
    if int(np.prod(shape)) != n:
        raise ValueError("cannot reshape array of size {} into shape {}".format(n, shape))
    new_split = kwargs.get("new_split", a.split)
    if new_split is not None and len(shape) == 0:
        new_split = None
    new_split = sanitize_axis(shape, new_split)
    if not a.is_distributed():
        t = a.larray.reshape(shape)
        out = DNDarray(t, shape, a.dtype, None, a.device, a.comm, True)
        return resplit(out, new_split) if new_split is not None and a.comm.is_distributed() else \
            DNDarray(t, shape, a.dtype, new_split, a.device, a.comm, True)
    src = a if a.split == 0 else resplit(a, 0)
    rowsize = int(np.prod(src.gshape[1:])) if src.ndim > 1 else 1
    counts = src.split_counts()
    flat = src.larray.reshape(-1)
    p = a.comm.size
    segs = []
    off = 0
    for r in range(p):
        segs.append([(off * rowsize, 0, counts[r] * rowsize)] if counts[r] else [])
        off += counts[r]
    # target: split 0 of the new shape (flat contiguous block per rank)
    out_rows = _chunk_counts(shape[0], p) if len(shape) else [0] * p
    out_rowsize = int(np.prod(shape[1:])) if len(shape) > 1 else 1
    flat_out = _segment_exchange(flat, 0, a.comm, segs, [c * out_rowsize for c in out_rows])
    local = flat_out.reshape([out_rows[a.comm.rank]] + list(shape[1:]))
    out = DNDarray(local, shape, a.dtype, 0, a.device, a.comm, True)
    if new_split != 0:
        out.resplit_(new_split)
    return out


def flatten(a: DNDarray) -> DNDarray:
    """Flattened copy (split 0 if distributed)."""
    if a.split is None:
        return DNDarray(a.larray.flatten(), (a.gnumel,), a.dtype, None, a.device, a.comm, True)
    return reshape(a, (a.gnumel,), new_split=0)


def ravel(a: DNDarray) -> DNDarray:
    """Flattened array (a view when possible)."""
    if not a.is_distributed():
        return DNDarray(a.larray.reshape(-1), (a.gnumel,), a.dtype, None if a.split is None else 0, a.device,
                        a.comm, True)
    if a.split == 0:
        counts = a.split_counts()
        return DNDarray(a.larray.reshape(-1), (a.gnumel,), a.dtype, 0, a.device, a.comm,
                        None if a.balanced is not True or a.ndim > 1 else True)
    return flatten(a)


def swapaxes(x: DNDarray, axis1: int, axis2: int) -> DNDarray:
    """Interchange two axes (the split axis moves with its data, no communication)."""
    axis1 = sanitize_axis(x.gshape, axis1)
    axis2 = sanitize_axis(x.gshape, axis2)
    perm = list(range(x.ndim))
    perm[axis1], perm[axis2] = perm[axis2], perm[axis1]
    from .linalg.basics import transpose

    return transpose(x, perm)


def moveaxis(x: DNDarray, source, destination) -> DNDarray:
    """Move axes to new positions."""
    src = sanitize_axis(x.gshape, tuple(source) if isinstance(source, (list, tuple)) else (source,))
    dst = sanitize_axis(x.gshape, tuple(destination) if isinstance(destination, (list, tuple)) else (destination,))
    if len(src) != len(dst):
        raise ValueError("source and destination arguments must have the same number of elements")
    order = [n for n in range(x.ndim) if n not in src]
    for d, s in sorted(zip(dst, src)):
        order.insert(d, s)
    from .linalg.basics import transpose

    return transpose(x, order)


# ---------------------------------------------------------------------------------------------
# reordering
# ---------------------------------------------------------------------------------------------
def flip(a: DNDarray, axis=None) -> DNDarray:
    """Reverse the order of elements along the given axes."""
    if axis is None:
        axis = tuple(range(a.ndim))
    axis = sanitize_axis(a.gshape, axis)
    axes = (axis,) if isinstance(axis, int) else axis
    t = torch.flip(a.larray, axes)
    if a.split is None or a.split not in axes or not a.is_distributed():
        return DNDarray(t, a.gshape, a.dtype, a.split, a.device, a.comm, a.balanced)
    n = a.gshape[a.split]
    bounds = _partition_bounds(a.split_counts())
    segs = [[(n - e, 0, e - s)] if e > s else [] for s, e in bounds]
    res = _segment_exchange(t, a.split, a.comm, segs, _chunk_counts(n, a.comm.size))
    return DNDarray(res, a.gshape, a.dtype, a.split, a.device, a.comm, True)


def fliplr(a: DNDarray) -> DNDarray:
    """Reverse the order of the columns (axis 1); a split along axis 1 moves blocks between mirrored ranks."""
    return flip(a, 1)


def flipud(a: DNDarray) -> DNDarray:
    """Reverse the order of the rows (axis 0); a split along axis 0 moves blocks between mirrored ranks."""
    return flip(a, 0)


def roll(x: DNDarray, shift, axis=None) -> DNDarray:
    """Roll elements along axes; along the split axis one exchange moves the wrapped segments."""
    if not isinstance(x, DNDarray):
        raise TypeError("expected x to be a ht.DNDarray, but was {}".format(type(x)))
    if axis is None:
        if not isinstance(shift, (int, np.integer)):
            raise TypeError("shift must be an integer when axis is None")
        flat = flatten(x)
        rolled = roll(flat, shift, 0)
        return reshape(rolled, x.gshape, new_split=x.split)
    if isinstance(axis, (list, tuple)):
        shifts = shift if isinstance(shift, (list, tuple)) else [shift] * len(axis)
        if len(shifts) != len(axis):
            raise ValueError("shift and axis length must match")
        res = x
        for s, ax in zip(shifts, axis):
            res = roll(res, s, ax)
        return res
    if isinstance(shift, (list, tuple)):
        res = x
        for s in shift:
            res = roll(res, s, axis)
        return res
    if not isinstance(shift, (int, np.integer)):
        raise TypeError("shift must be an integer or a sequence of integers")
    axis = sanitize_axis(x.gshape, axis)
    if not x.is_distributed() or axis != x.split:
        return DNDarray(torch.roll(x.larray, int(shift), axis), x.gshape, x.dtype, x.split, x.device, x.comm,
                        x.balanced)
    n = x.gshape[axis]
    k = int(shift) % n if n else 0
    bounds = _partition_bounds(x.split_counts())
    segs = []
    for s, e in bounds:
        rs = []
        if e > s:
            g = (s + k) % n
            first = min(e - s, n - g)
            rs.append((g, 0, first))
            if first < e - s:
                rs.append((0, first, e - s - first))
        segs.append(rs)
    res = _segment_exchange(x.larray, axis, x.comm, segs, _chunk_counts(n, x.comm.size))
    return DNDarray(res, x.gshape, x.dtype, x.split, x.device, x.comm, True)


def rot90(m: DNDarray, k: int = 1, axes: Sequence[int] = (0, 1)) -> DNDarray:
    """Rotate by 90 degrees in the plane of ``axes``."""
    axes = tuple(axes)
    if len(axes) != 2:
        raise ValueError("len(axes) must be 2.")
    if not isinstance(m, DNDarray):
        raise TypeError("expected m to be a ht.DNDarray, but was {}".format(type(m)))
    if axes[0] == axes[1] or np.absolute(axes[0] - axes[1]) == m.ndim:
        raise ValueError("Axes must be different.")
    if axes[0] >= m.ndim or axes[0] < -m.ndim or axes[1] >= m.ndim or axes[1] < -m.ndim:
        raise ValueError("Axes={} out of range for array of ndim={}.".format(axes, m.ndim))
    if not isinstance(k, (int, np.integer)):
        raise TypeError("Unknown type, must be int")
    k %= 4
    if k == 0:
        return m.copy()
    if k == 2:
        return flip(flip(m, axes[0]), axes[1])
    perm = list(range(m.ndim))
    perm[axes[0]], perm[axes[1]] = perm[axes[1]], perm[axes[0]]
    from .linalg.basics import transpose

    if k == 1:
        return transpose(flip(m, axes[1]), perm)
    return flip(transpose(m, perm), axes[1])


# ---------------------------------------------------------------------------------------------
# padding / repetition
# ---------------------------------------------------------------------------------------------
def pad(array: DNDarray, pad_width, mode: str = "constant", constant_values=0) -> DNDarray:
    """Constant padding (NumPy ``pad_width`` conventions); the result is balanced."""
    if not isinstance(array, DNDarray):
        raise TypeError("expected array to be a ht.DNDarray, but was {}".format(type(array)))
    if not isinstance(mode, str):
        raise TypeError("expected mode to be a string, but was {}".format(type(mode)))
    if mode != "constant":
        raise NotImplementedError("only mode='constant' is supported, got {}".format(mode))
    if not isinstance(pad_width, (int, tuple, list)):
        raise TypeError("expected pad_width to be an integer or a sequence (tuple or list), but was {}".format(
            type(pad_width)))
    nd = array.ndim
    if isinstance(pad_width, int):
        widths = [(pad_width, pad_width)] * nd
    else:
        pw = list(pad_width)
        if len(pw) and isinstance(pw[0], int):
            if len(pw) == 1:
                widths = [(pw[0], pw[0])] * nd
            elif len(pw) == 2 and nd != 1 or (nd == 1 and len(pw) == 2):
                widths = [(pw[0], pw[1])] * nd
            else:
                raise ValueError("invalid pad_width {}".format(pad_width))
        else:
            pw = [tuple(w) if isinstance(w, (list, tuple)) else (w, w) for w in pw]
            if len(pw) == 1:
                widths = [pw[0]] * nd
            elif len(pw) == nd:
                widths = pw
            else:
                # NumPy-like: pad_width for the last dims (torch convention) is not supported
                raise ValueError("pad_width must have one entry per dimension")
    widths = [(int(a), int(b)) for a, b in widths]
    for a, b in widths:
        if a < 0 or b < 0:
            raise ValueError("pad_width values must be non-negative")
    cv = constant_values
    if isinstance(cv, (list, tuple)):
        cvs = [tuple(c) if isinstance(c, (list, tuple)) else (c, c) for c in cv]
        if len(cvs) == 1:
            cvs = cvs * nd
    else:
        cvs = [(cv, cv)] * nd
    t = array.larray
    split = array.split if array.is_distributed() else None
    # pad every non-split axis locally, first axis first: a later (higher) axis pads the full
    # extent of the earlier ones, so corners take the higher axis' constant (NumPy)
    for ax in range(nd):
        if ax == split:
            continue
        before, after = widths[ax]
        if before == 0 and after == 0:
            continue
        parts = []
        if before:
            sh = list(t.shape)
            sh[ax] = before
            parts.append(torch.full(sh, cvs[ax][0], dtype=t.dtype, device=t.device))
        parts.append(t)
        if after:
            sh = list(t.shape)
            sh[ax] = after
            parts.append(torch.full(sh, cvs[ax][1], dtype=t.dtype, device=t.device))
        t = torch.cat(parts, dim=ax)
    gshape = tuple(s + widths[i][0] + widths[i][1] for i, s in enumerate(array.gshape))
    if split is None:
        return DNDarray(t, gshape, array.dtype, array.split, array.device, array.comm, True)
    before, after = widths[split]
    p, me = array.comm.size, array.comm.rank
    counts = array.split_counts()
    bounds = _partition_bounds(counts)
    # the first / last rank contributes the constant rows
    first = next((r for r in range(p) if counts[r] > 0), 0)
    last = max((r for r in range(p) if counts[r] > 0), default=p - 1)
    local_parts, segs = [], [[] for _ in range(p)]
    for r in range(p):
        lpos = 0
        if r == first and before:
            segs[r].append((0, lpos, before))
            lpos += before
        if counts[r]:
            segs[r].append((before + bounds[r][0], lpos, counts[r]))
            lpos += counts[r]
        if r == last and after:
            segs[r].append((before + array.gshape[split], lpos, after))
    if me == first and before:
        sh = list(t.shape)
        sh[split] = before
        local_parts.append(torch.full(sh, cvs[split][0], dtype=t.dtype, device=t.device))
    local_parts.append(t)
    if me == last and after:
        sh = list(t.shape)
        sh[split] = after
        local_parts.append(torch.full(sh, cvs[split][1], dtype=t.dtype, device=t.device))
    local = torch.cat(local_parts, dim=split)
    res = _segment_exchange(local, split, array.comm, segs, _chunk_counts(gshape[split], p))
    # the split-axis rows were filled with the split axis' constant everywhere; the pad regions of
    # higher axes win their corners (NumPy)
    for ax in range(split + 1, nd):
        before, after = widths[ax]
        if cvs[ax] == cvs[split] or res.numel() == 0:
            continue
        if before:
            res.narrow(ax, 0, before).fill_(cvs[ax][0])
        if after:
            res.narrow(ax, res.shape[ax] - after, after).fill_(cvs[ax][1])
    return DNDarray(res, gshape, array.dtype, split, array.device, array.comm, True)


def repeat(a, repeats, axis: Optional[int] = None) -> DNDarray:
    """Repeat elements (scalar or per-element ``repeats``); the result is balanced."""
    if not isinstance(a, DNDarray):
        a = factories.array(a)
    if isinstance(repeats, DNDarray):
        rep_t = repeats._gathered().to(torch.int64)
    elif isinstance(repeats, (list, tuple, np.ndarray)):
        rep_t = torch.as_tensor(np.asarray(repeats), dtype=torch.int64)
    elif isinstance(repeats, (int, np.integer)):
        rep_t = None
        if repeats < 0:
            raise ValueError("negative dimensions are not allowed")
    else:
        raise TypeError("repeats must be an int, list, tuple, ndarray or DNDarray, got {}".format(type(repeats)))
    if axis is None:
        a = flatten(a)
        axis = 0
    axis = sanitize_axis(a.gshape, axis)
    n = a.gshape[axis]
    if rep_t is not None and rep_t.numel() not in (1, n):
        raise ValueError("repeats must have the same length as the axis ({}), got {}".format(n, rep_t.numel()))
    if rep_t is not None and rep_t.numel() == 1:
        repeats, rep_t = int(rep_t.item()), None
    t = a.larray
    if a.is_distributed() and axis == a.split:
        counts, displs = a.counts_displs()
        me = a.comm.rank
        if rep_t is not None:
            local_rep = rep_t[displs[me]: displs[me] + counts[me]].to(t.device)
            res = torch.repeat_interleave(t, local_rep, dim=axis)
            new_counts = [int(rep_t[displs[r]: displs[r] + counts[r]].sum()) for r in range(a.comm.size)]
        else:
            res = torch.repeat_interleave(t, repeats, dim=axis)
            new_counts = [c * repeats for c in counts]
        gshape = list(a.gshape)
        gshape[axis] = sum(new_counts)
        out = DNDarray(res, tuple(gshape), a.dtype, a.split, a.device, a.comm, None)
        out.balance_()
        return out
    res = torch.repeat_interleave(t, rep_t.to(t.device) if rep_t is not None else repeats, dim=axis)
    gshape = list(a.gshape)
    gshape[axis] = res.shape[axis]
    return DNDarray(res, tuple(gshape), a.dtype, a.split, a.device, a.comm, a.balanced)


def tile(x: DNDarray, reps) -> DNDarray:
    """Construct an array by repeating ``x`` ``reps`` times (split-axis copies in one exchange)."""
    if not isinstance(x, DNDarray):
        raise TypeError("x must be a DNDarray")
    if isinstance(reps, (int, np.integer)):
        reps = (int(reps),)
    if not isinstance(reps, (list, tuple, np.ndarray)) or not all(isinstance(r, (int, np.integer)) for r in reps):
        raise TypeError("reps must be an integer or a sequence of integers, got {}".format(reps))
    reps = [int(r) for r in reps]
    if any(r < 0 for r in reps):
        raise ValueError("reps must be non-negative")
    nd = max(x.ndim, len(reps))
    reps = [1] * (nd - len(reps)) + reps
    if x.ndim < nd:
        x = reshape(x, (1,) * (nd - x.ndim) + tuple(x.gshape),
                    new_split=None if x.split is None else x.split + nd - x.ndim)
    gshape = tuple(s * r for s, r in zip(x.gshape, reps))
    if not x.is_distributed():
        return DNDarray(x.larray.repeat(*reps), gshape, x.dtype, x.split, x.device, x.comm, True)
    s = x.split
    local_reps = list(reps)
    local_reps[s] = 1
    t = x.larray.repeat(*local_reps)
    n = x.gshape[s]
    counts = x.split_counts()
    bounds = _partition_bounds(counts)
    segs = []
    for r in range(x.comm.size):
        rs = []
        if counts[r]:
            for k in range(reps[s]):
                rs.append((k * n + bounds[r][0], 0, counts[r]))
        segs.append(rs)
    res = _segment_exchange(t, s, x.comm, segs, _chunk_counts(gshape[s], x.comm.size))
    return DNDarray(res, gshape, x.dtype, s, x.device, x.comm, True)


# ---------------------------------------------------------------------------------------------
# diagonals
# ---------------------------------------------------------------------------------------------
def diagonal(a: DNDarray, offset: int = 0, dim1: int = 0, dim2: int = 1) -> DNDarray:
    """Diagonal of ``a`` over ``dim1``/``dim2``, appended as the last axis of the result."""
    if not isinstance(a, DNDarray):
        raise TypeError("expected a DNDarray, got {}".format(type(a)))
    if a.ndim < 2:
        raise ValueError("diagonal requires an array of at least 2 dimensions, got {}".format(a.ndim))
    if not isinstance(offset, (int, np.integer)) or isinstance(offset, bool):
        raise ValueError("offset must be an integer, got {}".format(type(offset)))
    offset = int(offset)
    dim1 = sanitize_axis(a.gshape, dim1)
    dim2 = sanitize_axis(a.gshape, dim2)
    if dim1 == dim2:
        raise ValueError("Dim1 and dim2 need to be different")
    if not a.is_distributed() or a.split not in (dim1, dim2):
        res = torch.diagonal(a.larray, offset=offset, dim1=dim1, dim2=dim2)
        gshape = list(torch.diagonal(a.__torch_proxy__(), offset, dim1, dim2).shape)
        split = None
        if a.split is not None:
            split = a.split - sum(1 for d in (dim1, dim2) if d < a.split)
        return DNDarray(res.contiguous(), tuple(gshape), a.dtype, split, a.device, a.comm, a.balanced)
    counts, displs = a.counts_displs()
    me = a.comm.rank
    off = displs[me]
    # local offset so that global diagonal element (i, i+offset) maps to local coordinates
    if a.split == dim1:
        loc_offset = offset + off
    else:
        loc_offset = offset - off
    res = torch.diagonal(a.larray, offset=loc_offset, dim1=dim1, dim2=dim2).contiguous()
    gshape = list(torch.diagonal(a.__torch_proxy__(), offset, dim1, dim2).shape)
    split = len(gshape) - 1
    out = DNDarray(res, tuple(gshape), a.dtype, split, a.device, a.comm, None)
    return out


def diag(a: DNDarray, offset: int = 0) -> DNDarray:
    """1-D -> diagonal matrix, 2-D -> its diagonal."""
    if not isinstance(a, DNDarray):
        raise TypeError("expected a DNDarray, got {}".format(type(a)))
    if not isinstance(offset, (int, np.integer)) or isinstance(offset, bool):
        raise ValueError("offset must be an integer, got {}".format(type(offset)))
    offset = int(offset)
    if len(a.gshape) > 1:
        return diagonal(a, offset=offset)
    if len(a.gshape) < 1:
        raise ValueError("input array must be of dimension 1 or greater")
    if not isinstance(offset, int):
        raise ValueError("offset must be an integer, got {}".format(type(offset)))
    n = a.gshape[0] + abs(offset)
    if not a.is_distributed():
        res = torch.diag(a.larray, offset)
        return DNDarray(res, (n, n), a.dtype, a.split, a.device, a.comm, True)
    # rank r builds its row block [R0, R1) of the n x n result; its diagonal entries are the
    # contiguous range v[R0 - max(-offset, 0) ...] of the vector: ONE redistribution of the vector
    # (O(local) memory), no gather
    comm = a.comm
    m = a.gshape[0]
    counts = [comm.chunk((n, n), 0, rank=r)[1][0] for r in range(comm.size)]
    starts = np.concatenate([[0], np.cumsum(counts)[:-1]]).astype(np.int64)
    sh = -offset if offset < 0 else 0   # row j holds v[j - sh]
    need = [max(0, min(m, s0 + c - sh) - max(0, s0 - sh)) for s0, c in zip(starts, counts)]
    v = a.copy()
    target = torch.tensor(need, dtype=torch.int64).reshape(-1, 1)
    v.redistribute_(lshape_map=v.create_lshape_map(), target_map=target)
    R0, R1 = int(starts[comm.rank]), int(starts[comm.rank] + counts[comm.rank])
    res = torch.zeros((R1 - R0, n), dtype=a.larray.dtype, device=a.larray.device)
    vl = v.larray
    if vl.numel():
        j0 = max(R0, sh)                                    # first row with an entry
        rows = torch.arange(j0 - R0, j0 - R0 + vl.shape[0], device=res.device)
        cols = torch.arange(j0 + offset, j0 + offset + vl.shape[0], device=res.device)
        res[rows, cols] = vl
    return DNDarray(res, (n, n), a.dtype, 0, a.device, comm, True)


# ---------------------------------------------------------------------------------------------
# splitting
# ---------------------------------------------------------------------------------------------
def split(x: DNDarray, indices_or_sections, axis: int = 0) -> List[DNDarray]:
    """Split into sub-arrays (views of the local blocks; split-axis pieces may be unbalanced)."""
    if not isinstance(x, DNDarray):
        raise TypeError("Expected x to be a DNDarray, but was {}".format(type(x)))
    axis = sanitize_axis(x.gshape, axis)
    n = x.gshape[axis]
    if isinstance(indices_or_sections, (int, np.integer)):
        k = int(indices_or_sections)
        if k <= 0 or n % k:
            raise ValueError("array split does not result in an equal division")
        bounds = [i * (n // k) for i in range(1, k)]
    elif isinstance(indices_or_sections, (list, tuple)):
        bounds = list(indices_or_sections)
    elif isinstance(indices_or_sections, DNDarray):
        bounds = indices_or_sections._gathered().tolist()
    elif isinstance(indices_or_sections, (np.ndarray, torch.Tensor)):
        bounds = list(np.asarray(indices_or_sections.cpu() if isinstance(indices_or_sections, torch.Tensor)
                                 else indices_or_sections).tolist())
    else:
        raise TypeError("indices_or_sections must be int, list, tuple, ndarray or DNDarray")
    edges = [0] + [min(max(int(b), 0), n) for b in bounds] + [n]
    out = []
    for i in range(len(edges) - 1):
        lo, hi = edges[i], max(edges[i], edges[i + 1])
        key = [slice(None)] * x.ndim
        key[axis] = slice(lo, hi)
        out.append(x[tuple(key)])
    return out


def hsplit(x: DNDarray, indices_or_sections) -> List[DNDarray]:
    """Split into sub-arrays along axis 1 (axis 0 for 1-D input), as ``split(x, indices_or_sections, 1)``."""
    if len(x.gshape) < 1:
        raise ValueError("hsplit only works on arrays of 1 or more dimensions")
    return split(x, indices_or_sections, axis=1 if x.ndim > 1 else 0)


def vsplit(x: DNDarray, indices_or_sections) -> List[DNDarray]:
    """Split into sub-arrays along axis 0 (input of 2 or more dimensions)."""
    if len(x.gshape) < 2:
        raise ValueError("vsplit only works on arrays of 2 or more dimensions")
    return split(x, indices_or_sections, axis=0)


def dsplit(x: DNDarray, indices_or_sections) -> List[DNDarray]:
    """Split into sub-arrays along axis 2 (input of 3 or more dimensions)."""
    if len(x.gshape) < 3:
        raise ValueError("dsplit only works on arrays of 3 or more dimensions")
    return split(x, indices_or_sections, axis=2)


# ---------------------------------------------------------------------------------------------
# sorting, selection, uniqueness
# ---------------------------------------------------------------------------------------------
def _desc_key(col: torch.Tensor) -> torch.Tensor:
    """Order-reversing involution used to sort descending with an ascending sort."""
    if col.dtype == torch.bool:
        return ~col
    if col.dtype == torch.uint8:
        return 255 - col
    if col.is_floating_point():
        return -col
    return ~col  # two's complement: ~x = -x - 1 reverses the order without overflow


def sort(a: DNDarray, axis: int = -1, descending: bool = False, out: Optional[DNDarray] = None):
    """Sort along ``axis``; returns ``(values, indices)`` (int64 global indices along ``axis``).

    Along the split axis: parallel sorting by regular sampling (local sort, p-1 samples per rank,
    pivot all-gather, one exchange of the partitions, local merge, one rebalancing exchange)."""
    if not isinstance(a, DNDarray):
        raise TypeError("expected a to be a DNDarray")
    axis = sanitize_axis(a.gshape, axis)
    if not a.is_distributed() or axis != a.split:
        vals, idx = _sample_sort.local_sort(a.larray, axis, descending)
        v = DNDarray(vals, a.gshape, a.dtype, a.split, a.device, a.comm, a.balanced)
        i = DNDarray(idx, a.gshape, types.int64, a.split, a.device, a.comm, a.balanced)
        if out is not None:
            out.larray = vals
            return i
        return v, i
    t = a.larray.movedim(axis, -1)
    lead = tuple(t.shape[:-1])
    counts, displs = a.counts_displs()
    me = a.comm.rank
    gidx = torch.arange(displs[me], displs[me] + counts[me], device=t.device, dtype=torch.int64)
    # the number of columns is the same on every rank (product of the non-split dims)
    ncols = int(np.prod([s for i, s in enumerate(a.gshape) if i != axis])) if a.ndim > 1 else 1
    cols = t.reshape(ncols, t.shape[-1])
    if cols.dtype == torch.bool:
        cols = cols.to(torch.uint8)
    n = a.gshape[axis]
    nloc = _chunk_counts(n, a.comm.size)[me]
    if ncols and n:
        # all columns in one batched sample sort (the order-reversing keys are involutions)
        v, i = _sample_sort.sort_columns(_desc_key(cols) if descending else cols, gidx, a.comm, n)
        v = _desc_key(v) if descending else v
    else:
        v = cols.new_empty((ncols, nloc))
        i = torch.empty((ncols, nloc), dtype=torch.int64, device=t.device)
    v = v.reshape(lead + (nloc,)).movedim(-1, axis).contiguous()
    i = i.reshape(lead + (nloc,)).movedim(-1, axis).contiguous()
    vd = DNDarray(v.to(a.larray.dtype), a.gshape, a.dtype, a.split, a.device, a.comm, True)
    idd = DNDarray(i, a.gshape, types.int64, a.split, a.device, a.comm, True)
    if out is not None:
        out.larray = vd.larray
        return idd
    return vd, idd


def unique(a: DNDarray, sorted: bool = False, return_inverse: bool = False, axis: Optional[int] = None):
    """Unique elements (replicated result); ``return_inverse`` gives indices into it."""
    if axis is None:
        local = torch.unique(a.larray, sorted=True)
        if a.is_distributed():
            allu = a.comm.allgather_tensor(local, 0)
            uniq = torch.unique(allu, sorted=True)
        else:
            uniq = local
        res = DNDarray(uniq, tuple(uniq.shape), a.dtype, None, a.device, a.comm, True)
        if return_inverse:
            inv = torch.searchsorted(uniq, a.larray.reshape(-1).contiguous()).reshape(a.larray.shape)
            inv_arr = DNDarray(inv, a.gshape, types.int64, a.split, a.device, a.comm, a.balanced)
            return res, inv_arr
        return res
    axis = sanitize_axis(a.gshape, axis)
    if not a.is_distributed():
        uniq, inv = torch.unique(a.larray, sorted=True, return_inverse=True, dim=axis)
        res = DNDarray(uniq, tuple(uniq.shape), a.dtype, None, a.device, a.comm, True)
        if return_inverse:
            return res, DNDarray(inv, tuple(inv.shape), types.int64, None, a.device, a.comm, True)
        return res
    # slices along `axis` must be whole on one rank: split the array along `axis` (one
    # redistribution when it is split elsewhere), unique the local slices, ONE all-gather of the
    # local uniques (not of the array), and unique again; the inverse of the local slices comes
    # from their position among the global uniques
    src = a if a.split == axis else resplit(a, axis)
    local_u = torch.unique(src.larray, sorted=True, dim=axis)
    allu = a.comm.allgather_tensor(local_u, axis)
    uniq = torch.unique(allu, sorted=True, dim=axis)
    res = DNDarray(uniq, tuple(uniq.shape), a.dtype, None, a.device, a.comm, True)
    if a.split is not None and a.split != axis:
        res = resplit(res, a.split)
    if return_inverse:
        nu = uniq.shape[axis]
        _, inv_all = torch.unique(torch.cat([uniq, src.larray], dim=axis), sorted=True, return_inverse=True,
                                  dim=axis)
        inv = inv_all[nu:]
        inv_arr = DNDarray(inv, (a.gshape[axis],), types.int64, 0, a.device, a.comm, src.balanced)
        return res, inv_arr
    return res


def topk(a: DNDarray, k: int, dim: int = -1, largest: bool = True, sorted: bool = True,
         out: Optional[Tuple[DNDarray, DNDarray]] = None):
    """The k largest (or smallest) entries along ``dim`` and their global indices.

    Along the split axis: local top-k, one all-gather of the p*k candidates, top-k of those
    (replaces the reference's custom MPI_TOPK reduction, manipulations.py:3997)."""
    dim = sanitize_axis(a.gshape, dim)
    if not a.is_distributed() or dim != a.split:
        native = ops.topk_rows(a.larray, k, dim, largest)   # one wave per row (csrc/select.hip)
        vals, idx = native if native is not None else torch.topk(a.larray, k, dim=dim, largest=largest,
                                                                 sorted=sorted)
        gshape = list(a.gshape)
        gshape[dim] = k
        v = DNDarray(vals, tuple(gshape), a.dtype, a.split, a.device, a.comm, a.balanced)
        i = DNDarray(idx, tuple(gshape), types.int64, a.split, a.device, a.comm, a.balanced)
    else:
        counts, displs = a.counts_displs()
        me = a.comm.rank
        kl = min(k, counts[me])
        native = ops.topk_rows(a.larray, kl, dim, largest, displs[me]) if kl > 0 else None
        if native is not None:
            vals, idx = native
        else:
            vals, idx = torch.topk(a.larray, kl, dim=dim, largest=largest, sorted=True)
            idx = idx + displs[me]
        # pad to k with sentinel values so every rank contributes k candidates
        if kl < k:
            sh = list(vals.shape)
            sh[dim] = k - kl
            if vals.is_floating_point():
                fill = -float("inf") if largest else float("inf")
            else:
                info = torch.iinfo(vals.dtype) if vals.dtype != torch.bool else None
                fill = (info.min if largest else info.max) if info else (not largest)
            vals = torch.cat([vals, torch.full(sh, fill, dtype=vals.dtype, device=vals.device)], dim=dim)
            idx = torch.cat([idx, torch.full(sh, -1, dtype=idx.dtype, device=idx.device)], dim=dim)
        allv = a.comm.allgather_tensor(vals.contiguous(), dim)
        alli = a.comm.allgather_tensor(idx.contiguous(), dim)
        v2, sel = torch.topk(allv, k, dim=dim, largest=largest, sorted=sorted)
        i2 = torch.gather(alli, dim, sel)
        gshape = list(a.gshape)
        gshape[dim] = k
        _, _, sl = a.comm.chunk(gshape, dim)
        v = DNDarray(v2[sl].contiguous(), tuple(gshape), a.dtype, dim, a.device, a.comm, True)
        i = DNDarray(i2[sl].contiguous(), tuple(gshape), types.int64, dim, a.device, a.comm, True)
    if out is not None:
        for o, r in zip(out, (v, i)):
            if o.gshape != r.gshape:
                raise ValueError("out shape {} does not match the result shape {}".format(o.gshape, r.gshape))
            if r.split != o.split:   # e.g. a replicated out buffer for a split-axis top-k
                r = resplit(r, o.split)
            if r.lshape != o.lshape:
                r = r.copy()
                r.redistribute_(lshape_map=r.create_lshape_map(), target_map=o.create_lshape_map())
            o.larray = r.larray.to(o.larray.dtype)
        return out
    return v, i


DNDarray.balance = lambda self: balance(self, copy=True)
DNDarray.expand_dims = lambda self, axis: expand_dims(self, axis)
DNDarray.flatten = lambda self: flatten(self)
DNDarray.redistribute = lambda self, lshape_map=None, target_map=None: redistribute(self, lshape_map, target_map)
DNDarray.reshape = lambda self, *shape, **kwargs: reshape(self, *shape, **kwargs)
DNDarray.resplit = lambda self, axis=None: resplit(self, axis)
DNDarray.rot90 = lambda self, k=1, axes=(0, 1): rot90(self, k, axes)
DNDarray.squeeze = lambda self, axis=None: squeeze(self, axis)
DNDarray.swapaxes = lambda self, axis1, axis2: swapaxes(self, axis1, axis2)
DNDarray.unique = lambda self, sorted=False, return_inverse=False, axis=None: unique(self, sorted, return_inverse, axis)



def mpi_topk(a, b, mpi_type=None) -> None:
    """Reduction callback of distributed :func:`topk` (reference manipulations.py:3997-4040):
    buffers are float64 ``[k, dim, largest, sorted, ndim, *shape, values..., indices...]``; the
    top-k of the concatenation of both candidate sets is written into ``b``."""
    ap = torch.as_tensor(a) if isinstance(a, torch.Tensor) else torch.from_numpy(np.frombuffer(a, dtype=np.float64))
    bp = torch.as_tensor(b) if isinstance(b, torch.Tensor) else torch.from_numpy(np.frombuffer(b, dtype=np.float64))
    k, dim, largest, srt = int(ap[0]), int(ap[1]), bool(ap[2]), bool(ap[3])
    la, lb = int(ap[4]), int(bp[4])
    sa = [int(v) for v in ap[5: 5 + la].tolist()]
    sb = [int(v) for v in bp[5: 5 + lb].tolist()]
    av, ai = ap[5 + la:].chunk(2)
    bv, bi = bp[5 + lb:].chunk(2)
    vals = torch.cat((av.reshape(sa), bv.reshape(sb)), dim=dim)
    idx = torch.cat((ai.reshape(sa), bi.reshape(sb)), dim=dim)
    res, kk = torch.topk(vals, k, dim=dim, largest=largest, sorted=srt)
    out = torch.cat((ap[: 5 + la], res.double().flatten(), torch.gather(idx, dim, kk).double().flatten()))
    bp.copy_(out)


MPI_TOPK = MPI.Op.Create(mpi_topk, commute=True)
