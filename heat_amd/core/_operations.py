"""
The split-aware operation engine: element-wise binary ops, element-wise local ops, reductions and
cumulative ops (reference ``heat/core/_operations.py``: ``__binary_op`` 25, ``__cum_op`` 184,
``__local_op`` 281, ``__reduce_op`` 355).

Split rules are the reference's: a replicated operand is sliced to the split operand's block
(``_operations.py:96-103``); reducing over the split axis yields ``split=None`` and a reduction
over a lower axis shifts the split down (``_operations.py:439-448``). Differences by design:

* operands split along different axes are aligned with one all-to-all instead of raising;
* unequally distributed operands along the same axis are aligned with one exchange;
* ``__cum_op`` carries the per-rank totals with one all-gather + local prefix (RCCL has no scan).
"""
from __future__ import annotations

import builtins
from typing import Callable, Optional, Sequence, Tuple, Union

import numpy as np
import torch

from . import devices, types
from .communication import MPI, Op
from .dndarray import DNDarray
from .stride_tricks import broadcast_shape, sanitize_axis

__all__ = []


def _scalar_tensor(v, device, dtype):
    return torch.tensor(v, device=device, dtype=dtype)


# torch ops that take a Python number as the second operand without changing the result type of an
# already-promoted tensor (the number rides in the kernel's arguments: no host-to-device copy of a
# 0-d tensor and no extra broadcast operand, ~35 us per call on the GPU)
_NUMBER_OK = {torch.add, torch.sub, torch.mul, torch.div, torch.true_divide, torch.floor_divide, torch.remainder,
              torch.fmod, torch.pow, torch.eq, torch.ne, torch.lt, torch.le, torch.gt, torch.ge}
_NUMBER_TYPES = {torch.float32, torch.float64, torch.int8, torch.int16, torch.int32, torch.int64, torch.uint8}


_INT_DIVS = {torch.div, torch.true_divide, torch.floor_divide, torch.remainder, torch.fmod}
# floating tensors: only where the number is used as-is. Torch's device division by a scalar
# multiplies by its reciprocal (x / 3.0 off by an ulp, x / 1e-40 -> inf) and pow by a scalar
# switches to special cases (sqrt, x*x*x), so those keep the correctly rounded 0-d tensor path
_FLOAT_NUMBER_OK = {torch.add, torch.sub, torch.mul, torch.eq, torch.ne, torch.lt, torch.le, torch.gt, torch.ge}


def _number_operand(operation, fn_kwargs, ptype, v) -> bool:
    """Whether the scalar second operand ``v`` may go to ``operation`` as a Python number: same
    result type and value as the 0-d tensor of type ``ptype`` (integers must fit ``ptype``; integer
    divisions keep the tensor, whose division by zero does not raise)."""
    if operation not in _NUMBER_OK or fn_kwargs or ptype not in _NUMBER_TYPES or isinstance(v, bool):
        return False
    if ptype.is_floating_point:
        return operation in _FLOAT_NUMBER_OK and isinstance(v, (int, float))
    if not isinstance(v, int) or operation in _INT_DIVS:
        return False
    info = torch.iinfo(ptype)
    return info.min <= v <= info.max


def _is_scalar(x) -> bool:
    return np.isscalar(x) or (isinstance(x, torch.Tensor) and x.dim() == 0 and not isinstance(x, DNDarray))


def _align_to(src: DNDarray, ref_counts, out_split_src: int) -> torch.Tensor:
    """Return src's local block redistributed so its split axis matches ``ref_counts``."""
    from .dndarray import _partition_bounds

    cur = src.split_counts()
    if cur == list(ref_counts):
        return src.larray
    return src._exchange_rows(cur, list(ref_counts))


def binary_op(operation: Callable, t1, t2, out: Optional[DNDarray] = None, where=True,
              fn_kwargs: Optional[dict] = None) -> DNDarray:
    """Element-wise ``operation(t1, t2)`` with NumPy broadcasting and heat split semantics."""
    fn_kwargs = fn_kwargs or {}
    if not isinstance(t1, DNDarray) and not _is_scalar(t1):
        # sequences are rejected like the reference (_operations.py:65-80); NumPy arrays and torch
        # tensors are promoted to (replicated) DNDarrays
        if isinstance(t1, (np.ndarray, torch.Tensor)):
            from .factories import array

            t1 = array(t1, device=t2.device if isinstance(t2, DNDarray) else None)
        else:
            raise TypeError("Only DNDarrays and numeric scalars are supported, but input was {}".format(type(t1)))
    if not isinstance(t2, DNDarray) and not _is_scalar(t2):
        # sequences are rejected like the reference (_operations.py:65-80); NumPy arrays and torch
        # tensors are promoted to (replicated) DNDarrays
        if isinstance(t2, (np.ndarray, torch.Tensor)):
            from .factories import array

            t2 = array(t2, device=t1.device if isinstance(t1, DNDarray) else None)
        else:
            raise TypeError("Only DNDarrays and numeric scalars are supported, but input was {}".format(type(t2)))
    if not isinstance(t1, DNDarray) and not isinstance(t2, DNDarray):
        from .factories import array

        t1 = array(t1)
    promoted = types.result_type(t1, t2)
    ptype = promoted.torch_type()

    if not isinstance(t1, DNDarray) or not isinstance(t2, DNDarray):
        arr = t1 if isinstance(t1, DNDarray) else t2
        dev = arr.larray.device
        a = t1.larray.to(ptype) if isinstance(t1, DNDarray) else _scalar_tensor(
            t1.item() if isinstance(t1, torch.Tensor) else t1, dev, ptype)
        if isinstance(t2, DNDarray):
            b = t2.larray.to(ptype)
        else:
            v2 = t2.item() if isinstance(t2, torch.Tensor) else t2
            if _number_operand(operation, fn_kwargs, ptype, v2) and isinstance(t1, DNDarray):
                b = v2.item() if isinstance(v2, np.generic) else v2
            else:
                b = _scalar_tensor(v2, dev, ptype)
        result = operation(a, b, **fn_kwargs)
        gshape, split, balanced = arr.gshape, arr.split, arr.balanced
        comm, device = arr.comm, arr.device
    else:
        gshape = broadcast_shape(t1.gshape, t2.gshape)
        nd = len(gshape)
        s1 = None if t1.split is None else t1.split + nd - t1.ndim
        s2 = None if t2.split is None else t2.split + nd - t2.ndim
        comm, device = t1.comm, t1.device
        # a split axis of extent 1 that is broadcast: replicate that operand
        if s1 is not None and t1.gshape[t1.split] == 1 and gshape[s1] != 1 and t1.is_distributed():
            t1 = _replicated(t1)
            s1 = None
        if s2 is not None and t2.gshape[t2.split] == 1 and gshape[s2] != 1 and t2.is_distributed():
            t2 = _replicated(t2)
            s2 = None
        if s1 is not None and s2 is not None and s1 != s2:
            from .manipulations import resplit

            if s1 - (nd - t2.ndim) >= 0:
                t2 = resplit(t2, s1 - (nd - t2.ndim))
                s2 = s1
            else:
                # t1's split axis is a broadcast (leading) axis of t2: replicate t2 (it is
                # smaller than the result), the s1 path below slices it where needed
                t2 = resplit(t2, None)
                s2 = None
        a, b = t1.larray, t2.larray
        split = s1 if s1 is not None else s2
        balanced = True
        if split is not None and comm.is_distributed():
            if s1 is not None and s2 is not None:
                balanced = t1.balanced
                c1, c2 = t1.split_counts(), t2.split_counts()
                if c1 != c2:
                    b = _align_to(t2, c1, s2)
            elif s1 is not None:
                balanced = t1.balanced
                # slice the replicated t2 to t1's block along the split (when not broadcast)
                d2 = split - (nd - t2.ndim)
                if d2 >= 0 and t2.gshape[d2] != 1:
                    counts, displs = t1.counts_displs()
                    r = comm.rank
                    b = b.narrow(d2, displs[r], counts[r])
            else:
                balanced = t2.balanced
                d1 = split - (nd - t1.ndim)
                if d1 >= 0 and t1.gshape[d1] != 1:
                    counts, displs = t2.counts_displs()
                    r = comm.rank
                    a = a.narrow(d1, displs[r], counts[r])
        if a.device != b.device:
            b = b.to(a.device)
        result = operation(a.to(ptype), b.to(ptype), **fn_kwargs)
    if not isinstance(result, torch.Tensor):
        result = torch.tensor(result, device=device.torch_device)
    rtype = types.canonical_heat_type(result.dtype)
    if out is not None:
        if not isinstance(out, DNDarray):
            raise TypeError("expected out to be None or a DNDarray, but was {}".format(type(out)))
        if tuple(out.gshape) != tuple(gshape):
            raise ValueError("Expecting output buffer of shape {}, got {}".format(gshape, out.shape))
        if out.split != split:
            raise ValueError("Expecting output buffer with split {}, got {}".format(split, out.split))
        if where is not True and where is not None:
            w = where.larray if isinstance(where, DNDarray) else where
            out.larray.copy_(torch.where(w, result.to(out.larray.dtype), out.larray))
        else:
            if out.larray.shape != result.shape:
                out.larray = result.to(out.larray.dtype)
            else:
                out.larray.copy_(result)
        return out
    res = DNDarray(result, tuple(gshape), rtype, split, device, comm, balanced)
    if where is not True and where is not None:
        # positions where `where` is False are left uninitialised in NumPy; we keep t1's values
        w = where.larray if isinstance(where, DNDarray) else where
        base = t1.larray if isinstance(t1, DNDarray) and t1.larray.shape == result.shape else torch.zeros_like(result)
        res.larray.copy_(torch.where(w, result, base.to(result.dtype)))
    return res


def _replicated(x: DNDarray) -> DNDarray:
    from .manipulations import resplit

    return resplit(x, None)


def local_op(operation: Callable, x: DNDarray, out: Optional[DNDarray] = None, no_cast: bool = False,
             **kwargs) -> DNDarray:
    """Element-wise unary op on the local block (no communication).

    Unless ``no_cast``, exact types are promoted to floating point first (float32, or float64 for
    64-bit integers) like NumPy's ufuncs."""
    if not isinstance(x, DNDarray):
        raise TypeError("expected x to be a DNDarray, but was {}".format(type(x)))
    if out is not None and not isinstance(out, DNDarray):
        raise TypeError("expected out to be None or a DNDarray, but was {}".format(type(out)))
    t = x.larray
    if not no_cast and not (t.is_floating_point() or t.is_complex()):
        t = t.to(types.promote_types(x.dtype, types.float32).torch_type())
    result = operation(t, **kwargs)
    if out is not None:
        if out.gshape != x.gshape:
            raise ValueError("Expecting output buffer of shape {}, got {}".format(x.gshape, out.shape))
        out.larray.copy_(result)
        return out
    return DNDarray(result, x.gshape, types.canonical_heat_type(result.dtype), x.split, x.device, x.comm, x.balanced)


def _reduce_local(partial_op: Callable, t: torch.Tensor, axis, keepdim: bool, **kwargs) -> torch.Tensor:
    if axis is None:
        return partial_op(t.reshape(-1), dim=0, keepdim=False, **kwargs) if t.dim() else partial_op(t.reshape(-1), dim=0, keepdim=False, **kwargs)
    if isinstance(axis, int):
        return partial_op(t, dim=axis, keepdim=keepdim, **kwargs)
    res = t
    for ax in sorted(axis, reverse=True):
        res = partial_op(res, dim=ax, keepdim=True, **kwargs)
    if not keepdim:
        for ax in sorted(axis, reverse=True):
            res = res.squeeze(ax)
    return res


def reduce_op(x: DNDarray, partial_op: Callable, reduction_op: Op, axis=None, out: Optional[DNDarray] = None,
              keepdim: bool = False, neutral=None, **kwargs) -> DNDarray:
    """Reduction: local ``partial_op`` then (if the split axis is reduced) one all-reduce.

    ``partial_op(tensor, dim=..., keepdim=...)`` must accept a single int ``dim``.
    """
    if not isinstance(x, DNDarray):
        raise TypeError("expected x to be a DNDarray, but was {}".format(type(x)))
    if out is not None and not isinstance(out, DNDarray):
        raise TypeError("expected out to be None or a DNDarray, but was {}".format(type(out)))
    axis = sanitize_axis(x.shape, axis)
    if isinstance(axis, tuple) and len(axis) == 1:
        axis = axis[0]
    split = x.split
    t = x.larray
    red_axes = None if axis is None else ((axis,) if isinstance(axis, int) else tuple(axis))
    if (split is not None and t.shape[split] == 0 and x.is_distributed()
            and (red_axes is None or split in red_axes)):
        # empty local block whose split axis is reduced: substitute neutral elements so the
        # all-reduce is correct (ref _operations.py:401 guards on `split in axis` the same way;
        # a reduction along another axis keeps the empty block and its (.., 0, ..) shape)
        shp = list(t.shape)
        shp[split] = 1
        fill = neutral if neutral is not None else 0
        t = torch.full(shp, fill, dtype=t.dtype, device=t.device)
    if x.ndim == 0:
        # a full reduction yields shape (1,) like the reference (_operations.py:416-417)
        partial = partial_op(t.reshape(1), dim=0, keepdim=False, **kwargs)
        gshape, out_split = (1,), None
    else:
        partial = _reduce_local(partial_op, t, axis, keepdim, **kwargs)
        if axis is None:
            gshape = tuple([1] * x.ndim) if keepdim else (1,)
            out_split = None
        else:
            axes = (axis,) if isinstance(axis, int) else axis
            if keepdim:
                gshape = tuple(1 if i in axes else s for i, s in enumerate(x.gshape))
            else:
                gshape = tuple(s for i, s in enumerate(x.gshape) if i not in axes)
            if split is None or split in axes:
                out_split = None
            else:
                out_split = split if keepdim else split - sum(1 for a in axes if a < split)
    reduced_split = split is not None and x.is_distributed() and (axis is None or split in (
        (axis,) if isinstance(axis, int) else axis))
    if reduced_split:
        partial = partial.contiguous()
        x.comm.Allreduce(MPI.IN_PLACE, partial, reduction_op)
    balanced = True if out_split is None else x.balanced
    if isinstance(partial, tuple):
        partial = partial[0]
    partial = partial.reshape(gshape) if partial.numel() == int(np.prod(gshape)) and out_split is None else partial
    res = DNDarray(partial, gshape, types.canonical_heat_type(partial.dtype), out_split, x.device, x.comm, balanced)
    if out is not None:
        if tuple(out.gshape) != tuple(gshape):
            raise ValueError("Expecting output buffer of shape {}, got {}".format(gshape, out.shape))
        if out.split != out_split and x.comm.size > 1:
            from .manipulations import resplit

            res = resplit(res, out.split)
        partial = res.larray
        out.larray = partial.to(out.larray.dtype) if out.larray.shape != partial.shape else out.larray.copy_(partial)
        return out
    return res


def cum_op(x: DNDarray, partial_op: Callable, exscan_op: Op, final_op: Callable, neutral, axis: int, dtype=None,
           out: Optional[DNDarray] = None) -> DNDarray:
    """Cumulative op along ``axis``: local prefix, then the carry of lower ranks (one all-gather)."""
    if axis is None:
        raise NotImplementedError("axis = None is not supported")
    axis = sanitize_axis(x.shape, axis)
    if dtype is not None:
        dtype = types.canonical_heat_type(dtype)
        t = x.larray.to(dtype.torch_type())
    else:
        t = x.larray
        if t.dtype == torch.bool:
            t = t.to(torch.int64)
    cum = partial_op(t, dim=axis)
    if x.is_distributed() and axis == x.split:
        n = cum.shape[axis]
        shp = list(cum.shape)
        shp[axis] = 1
        if n > 0:
            last = cum.narrow(axis, n - 1, 1).contiguous()
        else:
            last = torch.full(shp, neutral, dtype=cum.dtype, device=cum.device)
        carry = torch.full(shp, neutral, dtype=cum.dtype, device=cum.device)
        x.comm.Exscan(last, carry, exscan_op)
        if x.comm.rank > 0 and n > 0:
            cum = final_op(cum, carry)
    if out is not None:
        out.larray.copy_(cum)
        return out
    return DNDarray(cum, x.gshape, types.canonical_heat_type(cum.dtype), x.split, x.device, x.comm, x.balanced)


# names used by the reference's modules (kept for users who import the private engine)
__binary_op = binary_op
__local_op = local_op
__reduce_op = reduce_op
__cum_op = cum_op
