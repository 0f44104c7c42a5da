"""
Statistical functions (reference ``heat/core/statistics.py``: ``argmax/argmin`` 44/115, ``average``
187, ``bincount`` 319, ``cov`` 382, ``histc/histogram`` 457/514, ``kurtosis/skew`` 562/1456,
``max/min`` 616/941, ``maximum/minimum`` 675/1001, ``mean`` 726, ``median`` 844, ``percentile`` 1210,
``std`` 1501, ``var`` 1634).

Moments are computed in ONE pass (native ``moments.hip`` on the GPU: count, mean, M2 with a
Chan merge in fp64) and merged across ranks with ONE all-gather of the packed triples, instead of
the reference's p-sized all-reduce buffers followed by a Python merge loop
(``statistics.py:799-810, 1725-1737``). arg-reductions all-gather (value, index) pairs instead of
the custom ``MPI_ARGMAX`` callbacks (``statistics.py:1139-1207``).
"""
from __future__ import annotations

from builtins import max as _bmax
from typing import Optional, Tuple, Union

import numpy as np
import torch

from . import _operations, factories, types
from .communication import MPI
from .dndarray import DNDarray
from .stride_tricks import sanitize_axis
from .. import ops

__all__ = ["argmax", "argmin", "average", "bincount", "cov", "histc", "histogram", "kurtosis", "max", "maximum",
           "mean", "median", "min", "minimum", "percentile", "skew", "std", "var"]


# ---------------------------------------------------------------------------------------------
# moments engine
# ---------------------------------------------------------------------------------------------
def _moments(x: DNDarray, axis, final=None, ddof: int = 0):
    """Global (count, mean, M2) along ``axis`` as local torch tensors plus result metadata.

    Returns (res, gshape, split, balanced) where ``res`` is this rank's block of the result
    (replicated when the split axis is reduced): the (n, mean, M2) triple, or with ``final`` in
    ('mean', 'var', 'std') the value itself. Without a cross-rank merge that is ONE fused kernel
    launch on the device (``ops.moments``)."""
    axis = sanitize_axis(x.gshape, axis)
    if isinstance(axis, tuple):
        if len(axis) == 1:
            axis = axis[0]
        elif len(axis) == x.ndim:
            axis = None
        else:
            # several axes: move them to the end and flatten them into one
            keep = [i for i in range(x.ndim) if i not in axis]
            from .linalg.basics import transpose
            from .manipulations import reshape

            t = transpose(x, keep + list(axis))
            tail = int(np.prod([x.gshape[a] for a in axis]))
            newshape = tuple(x.gshape[i] for i in keep) + (tail,)
            new_split = None
            if x.split is not None:
                new_split = keep.index(x.split) if x.split in keep else len(keep)
            t = reshape(t, newshape, new_split=new_split)
            return _moments(t, len(keep), final, ddof)
    t = x.larray
    merge = x.is_distributed() and (axis is None or axis == x.split)
    if axis is None:
        gshape, split, bal = (), None, True
    else:
        gshape = tuple(s for i, s in enumerate(x.gshape) if i != axis)
        split, bal = None, True
        if not merge and x.split is not None and x.split != axis:
            split = x.split if x.split < axis else x.split - 1
            bal = x.balanced
    if not merge:
        return ops.moments(t, axis, final, ddof), gshape, split, bal
    n, mu, m2 = ops.moments(t, axis)
    n, mu, m2 = _allmerge(x.comm, n, mu, m2)
    if final is None:
        return (n, mu, m2), gshape, split, bal
    if final == "mean":
        return mu, gshape, split, bal
    v = m2 / (n - ddof)
    return (v.sqrt() if final == "std" else v), gshape, split, bal


# outputs up to this many elements are merged from an all-gather of every rank's triples (one
# collective, latency-bound); larger ones by two all-reduces (3 x out instead of p x 3 x out)
_ALLGATHER_MERGE_MAX = 4096


def _allmerge(comm, n, mu, m2):
    """Chan merge of every rank's (n, mean, M2) partials (fp64). Small outputs: ONE all-gather of
    the packed triples and a fixed-order merge. Large outputs: all-reduce [n, n mean] -> global
    mean, then all-reduce the M2 contributions around it (m2_r + n_r (mean_r - mean)^2) - exact
    Chan algebra, no cancellation, traffic independent of the number of ranks."""
    if n.numel() <= _ALLGATHER_MERGE_MAX:
        packed = torch.stack([n.reshape(-1), mu.reshape(-1), m2.reshape(-1)])  # [3, out]
        allp = comm.allgather_tensor(packed.unsqueeze(0).contiguous(), 0)       # [p, 3, out]
        N, MU, M2 = ops.merge_moments(allp[:, 0], allp[:, 1], allp[:, 2], 0)
        return N.reshape(n.shape), MU.reshape(mu.shape), M2.reshape(m2.shape)
    s = torch.stack([n.reshape(-1), (n * mu).reshape(-1)])
    comm.Allreduce(MPI.IN_PLACE, s, MPI.SUM)
    N = s[0]
    MU = s[1] / torch.where(N > 0, N, torch.ones_like(N))
    d = mu.reshape(-1) - MU
    M2 = m2.reshape(-1) + n.reshape(-1) * d * d
    comm.Allreduce(MPI.IN_PLACE, M2, MPI.SUM)
    return N.reshape(n.shape), MU.reshape(mu.shape), M2.reshape(m2.shape)


def _result_dtype(x: DNDarray):
    if types.heat_type_is_inexact(x.dtype):
        return x.dtype
    return types.promote_types(x.dtype, types.float32) if x.dtype is not types.int64 else types.float64


def _wrap(x: DNDarray, t: torch.Tensor, gshape, split, balanced, dtype=None):
    dtype = dtype if dtype is not None else types.canonical_heat_type(t.dtype)
    return DNDarray(t.to(dtype.torch_type()), tuple(gshape), dtype, split, x.device, x.comm, balanced)


def _moment_axis(x: DNDarray, axis):
    """Validate a mean/var axis like the reference (statistics.py:853-866): a str axis is a
    TypeError; tuples/lists with non-int or repeated entries, tensors and out-of-range axes are
    ValueErrors."""
    if axis is None:
        return None
    if isinstance(axis, torch.Tensor):
        raise ValueError("axis must be None, an int or a tuple of ints, not a tensor")
    if isinstance(axis, (list, tuple)):
        if not all(isinstance(a, (int, np.integer)) and not isinstance(a, bool) for a in axis):
            raise ValueError("axis entries must be ints, got {}".format(axis))
        axis = tuple(int(a) for a in axis)
        if len(set(a % _bmax(1, x.ndim) if -x.ndim <= a < x.ndim else a for a in axis)) != len(axis):
            raise ValueError("repeated axis in {}".format(axis))
        for a in axis:
            if not -x.ndim <= a < _bmax(1, x.ndim):
                raise ValueError("axis {} is out of bounds for {} dimensions".format(a, x.ndim))
        return axis
    if not isinstance(axis, (int, np.integer)) or isinstance(axis, bool):
        raise TypeError("axis must be None, int or tuple, but was {}".format(type(axis)))
    if not -x.ndim <= axis < _bmax(1, x.ndim):
        raise ValueError("axis {} is out of bounds for {} dimensions".format(axis, x.ndim))
    return int(axis)


def mean(x: DNDarray, axis=None) -> DNDarray:
    """Arithmetic mean (single pass + one all-gather of (n, mean, M2) triples when split)."""
    if not isinstance(x, DNDarray):
        raise TypeError("expected x to be a ht.DNDarray, but was {}".format(type(x)))
    axis = _moment_axis(x, axis)
    if types.heat_type_is_complexfloating(x.dtype):
        from . import arithmetics

        s = arithmetics.sum(x, axis=axis)
        cnt = x.gnumel / max(1, s.gnumel)
        return s / cnt
    mu, gshape, split, bal = _moments(x, axis, "mean")
    return _wrap(x, mu, gshape, split, bal, _result_dtype(x))


def var(x: DNDarray, axis=None, ddof: int = 0, **kwargs) -> DNDarray:
    """Variance with ``ddof`` delta degrees of freedom (``bessel=True`` -> ddof 1)."""
    if not isinstance(x, DNDarray):
        raise TypeError("expected x to be a ht.DNDarray, but was {}".format(type(x)))
    if "bessel" in kwargs:
        ddof = 1 if kwargs["bessel"] else 0
    if not isinstance(ddof, (int, np.integer)) or isinstance(ddof, bool):
        raise TypeError("ddof must be an integer, got {}".format(type(ddof)))
    if ddof < 0:
        raise ValueError("ddof must be non-negative, got {}".format(ddof))
    if ddof > 1:
        raise NotImplementedError("only ddof 0 and 1 are supported, got {}".format(ddof))
    axis = _moment_axis(x, axis)
    v, gshape, split, bal = _moments(x, axis, kwargs.pop("_final", "var"), ddof)
    return _wrap(x, v, gshape, split, bal, _result_dtype(x))


def std(x: DNDarray, axis=None, ddof: int = 0, **kwargs) -> DNDarray:
    """Standard deviation (square root of :func:`var`, fused into the same kernel)."""
    return var(x, axis, ddof, _final="std", **kwargs)


def _central_moment_sums(x: DNDarray, axis, powers=(2, 3, 4)):
    """Two-pass central moments: global mean, then sums of (x - mean)^k (one all-reduce)."""
    if axis is not None and (not isinstance(axis, (int, np.integer)) or isinstance(axis, bool)):
        raise TypeError("axis must be None or an int, got {}".format(type(axis)))
    sanitize_axis(x.gshape, axis)
    mu = mean(x, axis)
    t = x.larray.double()
    axis_s = sanitize_axis(x.gshape, axis)
    if axis_s is None:
        d = t - mu.larray.double()
        sums = torch.stack([(d ** k).sum() for k in powers])
        if x.is_distributed():
            x.comm.Allreduce(MPI.IN_PLACE, sums, MPI.SUM)
        n = float(x.gnumel)
        return n, sums, (), None, True
    m = mu.larray.double()
    if x.is_distributed() and axis_s != x.split and x.split is not None:
        # mu is split like the result: broadcast it against the local block
        pass
    d = t - m.unsqueeze(axis_s)
    sums = torch.stack([(d ** k).sum(dim=axis_s) for k in powers])
    if x.is_distributed() and axis_s == x.split:
        x.comm.Allreduce(MPI.IN_PLACE, sums, MPI.SUM)
    n = float(x.gshape[axis_s])
    return n, sums, mu.gshape, mu.split, mu.balanced


def skew(x: DNDarray, axis: Optional[int] = None, unbiased: bool = True) -> DNDarray:
    """Sample skewness (Fisher-Pearson; bias-corrected when ``unbiased``)."""
    n, s, gshape, split, bal = _central_moment_sums(x, axis, (2, 3))
    m2, m3 = s[0] / n, s[1] / n
    g1 = m3 / m2 ** 1.5
    if unbiased:
        g1 = g1 * (n * (n - 1)) ** 0.5 / (n - 2)
    return _wrap(x, g1, gshape, split, bal, _result_dtype(x))


def kurtosis(x: DNDarray, axis: Optional[int] = None, unbiased: bool = True, Fischer: bool = True) -> DNDarray:
    """Kurtosis (Fisher: excess, Pearson otherwise; bias-corrected when ``unbiased``)."""
    n, s, gshape, split, bal = _central_moment_sums(x, axis, (2, 4))
    m2, m4 = s[0] / n, s[1] / n
    g2 = m4 / m2 ** 2
    if unbiased:
        g2 = ((n + 1) * (g2 - 3) + 6) * (n - 1) / ((n - 2) * (n - 3)) + 3
    if Fischer:
        g2 = g2 - 3
    return _wrap(x, g2, gshape, split, bal, _result_dtype(x))


# ---------------------------------------------------------------------------------------------
# min / max
# ---------------------------------------------------------------------------------------------
def _neutral_max(t: torch.Tensor):
    if t.dtype == torch.bool:
        return 0
    if t.is_floating_point():
        return -float("inf")
    return torch.iinfo(t.dtype).min


def _neutral_min(t: torch.Tensor):
    if t.dtype == torch.bool:
        return 1
    if t.is_floating_point():
        return float("inf")
    return torch.iinfo(t.dtype).max


def max(x: DNDarray, axis=None, out: Optional[DNDarray] = None, keepdim: Optional[bool] = None) -> DNDarray:
    """Maximum along ``axis`` (all-reduce MAX when the split axis is reduced)."""
    def _max(t, dim, keepdim):
        return torch.amax(t, dim=dim, keepdim=keepdim)

    return _operations.reduce_op(x, _max, MPI.MAX, axis=axis, out=out, neutral=_neutral_max(x.larray),
                                 keepdim=bool(keepdim))


def min(x: DNDarray, axis=None, out: Optional[DNDarray] = None, keepdim: Optional[bool] = None) -> DNDarray:
    """Minimum along ``axis`` (all-reduce MIN when the split axis is reduced)."""
    def _min(t, dim, keepdim):
        return torch.amin(t, dim=dim, keepdim=keepdim)

    return _operations.reduce_op(x, _min, MPI.MIN, axis=axis, out=out, neutral=_neutral_min(x.larray),
                                 keepdim=bool(keepdim))


def maximum(x1, x2, out: Optional[DNDarray] = None) -> DNDarray:
    """Element-wise maximum (NaN propagates)."""
    return _operations.binary_op(torch.maximum, x1, x2, out)


def minimum(x1, x2, out: Optional[DNDarray] = None) -> DNDarray:
    """Element-wise minimum (NaN propagates)."""
    return _operations.binary_op(torch.minimum, x1, x2, out)


def _argext(x: DNDarray, axis, out, largest: bool, keepdim: bool = False):
    if not isinstance(x, DNDarray):
        raise TypeError("axis must be None or an int, but was {}".format(type(x)))
    if axis is not None and not isinstance(axis, (int, np.integer)):
        raise TypeError("axis must be None or an int, but was {}".format(type(axis)))
    axis = sanitize_axis(x.gshape, axis)
    if out is not None and (not isinstance(out, DNDarray) or out.dtype is not types.int64):
        raise TypeError("out must be an int64 DNDarray, got {}".format(getattr(out, "dtype", type(out))))
    t = x.larray
    fn = torch.argmax if largest else torch.argmin
    if t.is_cuda and x.gnumel and ops.argreduce_supported(t, x.gnumel if axis is None else x.gshape[axis]):
        r = _argext_native(x, axis, largest, keepdim)
    elif axis is None:
        if x.is_distributed():
            counts, displs = x.counts_displs()
            me = x.comm.rank
            if t.numel():
                li = int(fn(t.reshape(-1)))
                val = t.reshape(-1)[li].to(torch.float64)
                coords = list(np.unravel_index(li, t.shape))
                coords[x.split] += displs[me]
                gi = int(np.ravel_multi_index(coords, x.gshape))
                has = 1.0
            else:
                val = torch.tensor(0.0, dtype=torch.float64, device=t.device)
                gi, has = 0, 0.0
            pack = torch.stack([val.reshape(()).to(torch.float64),
                                torch.tensor(float(gi), dtype=torch.float64, device=t.device),
                                torch.tensor(has, dtype=torch.float64, device=t.device)]).unsqueeze(0)
            allp = x.comm.allgather_tensor(pack, 0).cpu()
            best = None
            for r in range(allp.shape[0]):
                v, i, h = allp[r].tolist()
                if h == 0:
                    continue
                if best is None or (v > best[0] if largest else v < best[0]) or (v == best[0] and i < best[1]) \
                        or (v != v and not (best[0] != best[0])):
                    best = (v, i)
            res = torch.tensor(int(best[1]), dtype=torch.int64, device=t.device)
        else:
            res = fn(t.reshape(-1))
        gshape = (1,) * x.ndim if keepdim else (1,)
        res = res.reshape(gshape)
        r = DNDarray(res, gshape, types.int64, None, x.device, x.comm, True)
    elif x.is_distributed() and axis == x.split:
        counts, displs = x.counts_displs()
        me = x.comm.rank
        if t.shape[axis]:
            vals, idx = (torch.max if largest else torch.min)(t, dim=axis, keepdim=True)
            idx = idx + displs[me]
        else:
            shp = list(t.shape)
            shp[axis] = 1
            fill = _neutral_max(t) if largest else _neutral_min(t)
            vals = torch.full(shp, fill, dtype=t.dtype, device=t.device)
            idx = torch.full(shp, -1, dtype=torch.int64, device=t.device)
        allv = x.comm.allgather_tensor(vals.contiguous(), axis)
        alli = x.comm.allgather_tensor(idx.contiguous(), axis)
        # first occurrence wins: argmax over the rank-ordered candidates picks the lowest index
        sel = fn(allv, dim=axis, keepdim=True)
        res = torch.gather(alli, axis, sel)
        gshape = tuple(1 if i == axis else s for i, s in enumerate(x.gshape))
        if not keepdim:
            res = res.squeeze(axis)
            gshape = tuple(s for i, s in enumerate(x.gshape) if i != axis)
        r = DNDarray(res, gshape, types.int64, None, x.device, x.comm, True)
    else:
        res = fn(t, dim=axis, keepdim=keepdim)
        if keepdim:
            gshape = tuple(1 if i == axis else s for i, s in enumerate(x.gshape))
            split = x.split
        else:
            gshape = tuple(s for i, s in enumerate(x.gshape) if i != axis)
            split = None if x.split in (None, axis) else (x.split if x.split < axis else x.split - 1)
        r = DNDarray(res, gshape, types.int64, split, x.device, x.comm, x.balanced)
    if out is not None:
        out.larray = r.larray
        return out
    return r


def _argext_native(x: DNDarray, axis, largest: bool, keepdim: bool) -> DNDarray:
    """Device arg-reduction through packed (value, first index) int64 keys (``csrc/select.hip``):
    one local kernel, and along the split axis ONE int64 MAX all-reduce of the keys (the
    reference all-reduces a pickled custom op, statistics.py:1139-1207)."""
    t = x.larray
    dist_split = x.is_distributed()
    displ = x.counts_displs()[1][x.comm.rank] if dist_split else 0
    if axis is None:
        keys = ops.argreduce_keys(t, None, not largest, displ, x.gshape[x.split] if dist_split else None,
                                   x.split if dist_split else None)
        if dist_split:
            x.comm.Allreduce(MPI.IN_PLACE, keys, MPI.MAX)
        gshape = (1,) * x.ndim if keepdim else (1,)
        res = ops.argreduce_decode(keys).reshape(gshape)
        return DNDarray(res, gshape, types.int64, None, x.device, x.comm, True)
    along_split = dist_split and axis == x.split
    keys = ops.argreduce_keys(t, axis, not largest, displ if along_split else 0)
    if along_split:
        x.comm.Allreduce(MPI.IN_PLACE, keys, MPI.MAX)
    res = ops.argreduce_decode(keys)
    if keepdim:
        res = res.unsqueeze(axis)
        gshape = tuple(1 if i == axis else s for i, s in enumerate(x.gshape))
    else:
        gshape = tuple(s for i, s in enumerate(x.gshape) if i != axis)
    if along_split or x.split is None or x.split == axis:
        return DNDarray(res, gshape, types.int64, None, x.device, x.comm, True)
    split = x.split if (keepdim or x.split < axis) else x.split - 1
    return DNDarray(res, gshape, types.int64, split, x.device, x.comm, x.balanced)


def argmax(x: DNDarray, axis: Optional[int] = None, out: Optional[DNDarray] = None, **kwargs) -> DNDarray:
    """Indices of the maxima (first occurrence) along ``axis`` (flattened index if None)."""
    return _argext(x, axis, out, True, kwargs.get("keepdim", False))


def argmin(x: DNDarray, axis: Optional[int] = None, out: Optional[DNDarray] = None, **kwargs) -> DNDarray:
    """Indices of the minima (first occurrence) along ``axis`` (flattened index if None)."""
    return _argext(x, axis, out, False, kwargs.get("keepdim", False))


# ---------------------------------------------------------------------------------------------
# weighted / counting statistics
# ---------------------------------------------------------------------------------------------
def average(x: DNDarray, axis=None, weights: Optional[DNDarray] = None, returned: bool = False):
    """Weighted average along ``axis``."""
    from . import arithmetics

    if not isinstance(x, DNDarray):
        raise TypeError("expected x to be a ht.DNDarray, but was {}".format(type(x)))
    if weights is None:
        result = mean(x, axis)
        if returned:
            cnt = x.gnumel / max(1, result.gnumel)
            return result, factories.full_like(result, cnt)
        return result
    if not isinstance(weights, DNDarray):
        raise TypeError("weights must be a DNDarray, got {}".format(type(weights)))
    if weights.gshape != x.gshape:
        if axis is None:
            raise TypeError("Axis must be specified when shapes of x and weights differ.")
        if isinstance(axis, tuple):
            raise NotImplementedError("Weighted average over tuple axis not implemented yet.")
        if weights.ndim != 1:
            raise TypeError("1D weights expected when shapes of x and weights differ.")
        if weights.gshape[0] != x.gshape[axis]:
            raise ValueError("Length of weights not compatible with specified axis.")
        shp = [1] * x.ndim
        shp[axis] = weights.gshape[0]
        from .manipulations import reshape, resplit

        wsplit = axis if (x.split == axis) else None
        w = resplit(weights, None) if weights.split is not None else weights
        w = reshape(w, tuple(shp), new_split=None)
        if wsplit is not None:
            w = resplit(w, axis)
    else:
        if weights.split != x.split:
            raise NotImplementedError("weights of x's shape must have x's split {}, got {}".format(
                x.split, weights.split))
        w = weights
    wsum = arithmetics.sum(w, axis=axis) if w.gshape == x.gshape else None
    num = arithmetics.sum(x * w, axis=axis)
    if wsum is None:
        from .manipulations import squeeze

        wsum = arithmetics.sum(w, axis=axis)
        if wsum.gnumel == 1:
            wsum = float(wsum.item())
    if isinstance(wsum, DNDarray):
        from . import logical

        if logical.any(wsum == 0):
            raise ZeroDivisionError("Weights sum to zero, can't be normalized")
    elif wsum == 0:
        raise ZeroDivisionError("Weights sum to zero, can't be normalized")
    result = num / wsum
    if returned:
        if not isinstance(wsum, DNDarray) or wsum.gshape != result.gshape:
            wsum = factories.full(result.gshape, float(wsum.item() if isinstance(wsum, DNDarray) else wsum),
                                  dtype=result.dtype, split=result.split, device=result.device, comm=result.comm)
        return result, wsum
    return result


def bincount(x: DNDarray, weights: Optional[DNDarray] = None, minlength: int = 0) -> DNDarray:
    """Occurrences of each value in a non-negative int array (one MAX + one SUM all-reduce)."""
    if not isinstance(x, DNDarray):
        raise TypeError("x must be a DNDarray")
    if x.ndim != 1:
        raise ValueError("bincount expects a 1-D array, got {} dimensions".format(x.ndim))
    t = x.larray.reshape(-1).to(torch.int64)
    mx = int(t.max()) + 1 if t.numel() else 0
    length = builtins_max(mx, minlength)
    if x.is_distributed():
        length = x.comm.allreduce(length, MPI.MAX)
    w = None
    if weights is not None:
        if weights.gshape != x.gshape:
            raise ValueError("weights and x must have the same shape")
        if weights.split != x.split:
            raise ValueError("weights and x must have the same split")
        if weights.lshape != x.lshape:   # same split, another partition (e.g. x unbalanced)
            weights = weights.copy()
            weights.redistribute_(lshape_map=weights.create_lshape_map(), target_map=x.create_lshape_map())
        w = weights.larray.reshape(-1)
    counts = torch.bincount(t, weights=None if w is None else w.to(torch.float64), minlength=length)
    # an empty local block must agree with the others on dtype (float64 with weights, like NumPy)
    counts = counts.to(torch.int64 if w is None else torch.float64)
    if x.is_distributed():
        counts = counts.contiguous()
        x.comm.Allreduce(MPI.IN_PLACE, counts, MPI.SUM)
    return DNDarray(counts, tuple(counts.shape), types.canonical_heat_type(counts.dtype), None, x.device, x.comm, True)


def builtins_max(a, b):
    return a if a > b else b


def histc(input: DNDarray, bins: int = 100, min: int = 0, max: int = 0, out: Optional[DNDarray] = None) -> DNDarray:
    """Histogram with ``bins`` equal-width bins over [min, max] (data range when both are 0)."""
    lo, hi = float(min), float(max)
    t = input.larray
    if lo == hi:
        lo = float(globals()["min"](input).item())
        hi = float(globals()["max"](input).item())
    tt = t if t.is_floating_point() else t.float()
    hist = torch.histc(tt.reshape(-1), bins=bins, min=lo, max=hi)
    if input.is_distributed():
        hist = hist.contiguous()
        input.comm.Allreduce(MPI.IN_PLACE, hist, MPI.SUM)
    res = DNDarray(hist, tuple(hist.shape), types.canonical_heat_type(hist.dtype), None, input.device, input.comm,
                   True)
    if out is not None:
        out.larray = hist.to(out.larray.dtype)
        return out
    return res


def histogram(a: DNDarray, bins: int = 10, range: Tuple[int, int] = (0, 0), normed: Optional[bool] = None,
              weights: Optional[DNDarray] = None, density: Optional[bool] = None):
    """Histogram of ``a`` (like the reference: counts only, via :func:`histc`)."""
    if not isinstance(bins, int):
        raise NotImplementedError("bins must be an integer")
    if normed is not None:
        raise NotImplementedError("'normed' is not supported")
    if weights is not None:
        raise NotImplementedError("'weights' are not supported")
    if density:
        raise NotImplementedError("'density' is not supported")
    return histc(a, bins=bins, min=range[0], max=range[1])


# ---------------------------------------------------------------------------------------------
# order statistics
# ---------------------------------------------------------------------------------------------
def _interp(lo_v, hi_v, frac, interpolation):
    if interpolation == "linear":
        return lo_v + (hi_v - lo_v) * frac
    if interpolation == "lower":
        return lo_v
    if interpolation == "higher":
        return hi_v
    if interpolation == "midpoint":
        return (lo_v + hi_v) / 2
    if interpolation == "nearest":
        # numpy: round half to even on the fractional position
        return torch.where(frac > 0.5, hi_v, torch.where(frac < 0.5, lo_v, lo_v))
    raise ValueError("Invalid interpolation method {}".format(interpolation))


def percentile(x: DNDarray, q, axis: Optional[int] = None, out: Optional[DNDarray] = None,
               interpolation: str = "linear", keepdim: bool = False) -> DNDarray:
    """q-th percentile(s) along ``axis`` (distributed sort along the split axis)."""
    from .manipulations import flatten, sort

    if not isinstance(x, DNDarray):
        raise TypeError("expected x to be a ht.DNDarray, but was {}".format(type(x)))
    if isinstance(q, np.ndarray):
        raise TypeError("q must be a scalar, list, tuple or DNDarray, got a NumPy array")
    if out is not None and not isinstance(out, DNDarray):
        raise TypeError("out must be a DNDarray, got {}".format(type(out)))
    if interpolation not in ("linear", "lower", "higher", "midpoint", "nearest"):
        raise ValueError("Invalid interpolation method {}".format(interpolation))
    scalar_q = np.isscalar(q) or (isinstance(q, DNDarray) and q.ndim == 0)
    if isinstance(q, DNDarray):
        qv = q._gathered().double().reshape(-1).tolist()
    elif isinstance(q, torch.Tensor):
        qv = q.double().reshape(-1).tolist()
    else:
        qv = np.atleast_1d(np.asarray(q, dtype=np.float64)).tolist()
    for v in qv:
        if v < 0 or v > 100:
            raise ValueError("Percentiles must be in the range [0, 100], got {}".format(v))
    if axis is None:
        src = flatten(x) if x.ndim != 1 else x
        ax = 0
    else:
        if isinstance(axis, (list, tuple)):
            raise NotImplementedError("percentile over several axes is not supported")
        src = x
        ax = sanitize_axis(x.gshape, axis)
    n = src.gshape[ax]
    rdtype = _result_dtype(x)
    tdt = torch.float64 if rdtype is types.float64 else torch.float32
    if src.is_distributed() and ax == src.split:
        vals, _ = sort(src, axis=ax)
        positions = []
        for v in qv:
            pos = v / 100.0 * (n - 1)
            positions.append((int(np.floor(pos)), int(np.ceil(pos)), pos - np.floor(pos)))
        need = sorted(set([p for lo, hi, _ in positions for p in (lo, hi)]))
        idx = torch.tensor(need, dtype=torch.int64)
        key = [slice(None)] * vals.ndim
        key[ax] = idx
        picked = vals[tuple(key)]._gathered()
        where = {p: i for i, p in enumerate(need)}
        res = []
        for lo, hi, frac in positions:
            lo_v = picked.narrow(ax, where[lo], 1).squeeze(ax).to(tdt)
            hi_v = picked.narrow(ax, where[hi], 1).squeeze(ax).to(tdt)
            if interpolation == "nearest":
                # NumPy rounds a half position to the even index
                res.append(hi_v if frac > 0.5 or (frac == 0.5 and hi % 2 == 0) else lo_v)
                continue
            res.append(_interp(lo_v, hi_v, torch.tensor(frac, dtype=tdt, device=lo_v.device), interpolation))
        r = torch.stack(res)
        split = None
    else:
        t = src.larray.to(tdt)
        # q / 100 on the host: a device division by a scalar is a multiply by its reciprocal, which
        # moves e.g. 95 / 100 one ulp up and flips "nearest" at a half position (28.5 -> 29 for n = 31)
        qt = torch.tensor([v / 100.0 for v in qv], dtype=tdt, device=t.device)
        r = torch.quantile(t, qt, dim=ax, interpolation=interpolation) if t.numel() else \
            torch.empty((len(qv),) + tuple(s for i, s in enumerate(t.shape) if i != ax), dtype=tdt, device=t.device)
        split = None
        if src.split is not None and src.is_distributed():
            split = (src.split if src.split < ax else src.split - 1) + 1
    gshape = (len(qv),) + tuple(s for i, s in enumerate(src.gshape) if i != ax)
    if keepdim and axis is not None:
        r = r.unsqueeze(ax + 1)
        gshape = gshape[: ax + 1] + (1,) + gshape[ax + 1:]
        if split is not None and split > ax:
            split += 1
    elif keepdim and axis is None:
        r = r.reshape((len(qv),) + (1,) * x.ndim)
        gshape = (len(qv),) + (1,) * x.ndim
    if scalar_q:
        r = r[0]
        gshape = gshape[1:]
        split = None if split is None else split - 1
    res = DNDarray(r.to(rdtype.torch_type()).contiguous(), gshape, rdtype, split, x.device, x.comm,
                   True if split is None else src.balanced)
    if out is not None:
        if out.dtype is not rdtype:
            raise TypeError("out must have dtype {}, got {}".format(rdtype, out.dtype))
        if tuple(out.gshape) != tuple(gshape):
            raise ValueError("out must have shape {}, got {}".format(gshape, out.gshape))
        if out.split != split:
            raise ValueError("out must have split {}, got {}".format(split, out.split))
        out.larray = res.larray
        return out
    return res


def median(x: DNDarray, axis: Optional[int] = None, keepdim: bool = False) -> DNDarray:
    """Median along ``axis`` (50th percentile, linear interpolation)."""
    return percentile(x, 50.0, axis=axis, keepdim=keepdim)


def cov(m: DNDarray, y: Optional[DNDarray] = None, rowvar: bool = True, bias: bool = False,
        ddof: Optional[int] = None) -> DNDarray:
    """Covariance matrix (variables in rows when ``rowvar``); one distributed GEMM."""
    from . import arithmetics
    from .linalg.basics import matmul, transpose
    from .manipulations import concatenate

    from .manipulations import expand_dims

    if ddof is not None and not isinstance(ddof, int):
        raise TypeError("ddof must be integer")
    if not isinstance(m, DNDarray):
        raise TypeError("m must be a DNDarray")
    if y is not None and not isinstance(y, DNDarray):
        raise TypeError("y must be None or a DNDarray")
    if m.ndim > 2:
        raise ValueError("m has more than 2 dimensions")
    if y is not None and y.ndim > 2:
        raise ValueError("y has more than 2 dimensions")
    # NumPy semantics: a 1-D m or y is one variable (a row), whatever rowvar says
    x = expand_dims(m, 0) if m.ndim == 1 else (m if rowvar or m.gshape[0] == 1 else transpose(m))
    if y is not None:
        yy = expand_dims(y, 0) if y.ndim == 1 else (y if rowvar or y.gshape[0] == 1 else transpose(y))
        if yy.gshape[1] != x.gshape[1]:
            raise RuntimeError("m and y must have the same number of observations")
        x = concatenate([x, yy], axis=0)
    if not types.heat_type_is_inexact(x.dtype):
        x = x.astype(types.float64)
    if ddof is None:
        ddof = 0 if bias else 1
    n = x.gshape[1]
    if ddof > n:
        raise ValueError("ddof {} must not exceed the number of observations {}".format(ddof, n))
    avg = mean(x, axis=1)
    xc = x - expand_dims(avg, 1)
    c = matmul(xc, transpose(xc))
    c = c / float(n - ddof)
    return c


DNDarray.argmax = lambda self, axis=None, out=None, **kwargs: argmax(self, axis, out, **kwargs)
DNDarray.argmin = lambda self, axis=None, out=None, **kwargs: argmin(self, axis, out, **kwargs)
DNDarray.average = lambda self, axis=None, weights=None, returned=False: average(self, axis, weights, returned)
DNDarray.kurtosis = lambda self, axis=None, unbiased=True, Fischer=True: kurtosis(self, axis, unbiased, Fischer)
DNDarray.max = lambda self, axis=None, out=None, keepdim=None: max(self, axis, out, keepdim)
DNDarray.mean = lambda self, axis=None: mean(self, axis)
DNDarray.median = lambda self, axis=None, keepdim=False: median(self, axis, keepdim)
DNDarray.min = lambda self, axis=None, out=None, keepdim=None: min(self, axis, out, keepdim)
DNDarray.skew = lambda self, axis=None, unbiased=True: skew(self, axis, unbiased)
DNDarray.std = lambda self, axis=None, ddof=0, **kwargs: std(self, axis, ddof, **kwargs)
DNDarray.var = lambda self, axis=None, ddof=0, **kwargs: var(self, axis, ddof, **kwargs)


# --------------------------------------------------------------------------------------------
# packed (value, index) reduction operators (reference statistics.py:1139-1207). The buffers hold
# [values..., indices...] (float64); ties keep the smaller global index. They are Op callbacks
# ``f(in, inout, datatype)`` usable with ``comm.Allreduce(..., MPI_ARGMAX)``; argmax/argmin use the
# same rule on all-gathered candidates.
# --------------------------------------------------------------------------------------------
def _as_f64(buf) -> torch.Tensor:
    if isinstance(buf, torch.Tensor):
        return buf
    return torch.from_numpy(np.frombuffer(buf, dtype=np.float64))


def _arg_combine(a, b, larger: bool) -> None:
    lhs, rhs = _as_f64(a), _as_f64(b)
    vl, il = lhs.chunk(2)
    vr, ir = rhs.chunk(2)
    take_l = (vl > vr) if larger else (vl < vr)
    take_l = take_l | ((vl == vr) & (il < ir))
    rhs.copy_(torch.cat([torch.where(take_l, vl, vr), torch.where(take_l, il, ir)]))


def mpi_argmax(a, b, _=None) -> None:
    """Combine two packed (values, indices) buffers into ``b`` keeping the larger value."""
    _arg_combine(a, b, True)


def mpi_argmin(a, b, _=None) -> None:
    """Combine two packed (values, indices) buffers into ``b`` keeping the smaller value."""
    _arg_combine(a, b, False)


MPI_ARGMAX = MPI.Op.Create(mpi_argmax, commute=True)
MPI_ARGMIN = MPI.Op.Create(mpi_argmin, commute=True)
