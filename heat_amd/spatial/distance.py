"""
Pairwise distances between the rows of two DNDarrays (reference ``heat/spatial/distance.py``:
metrics 16-133, ``cdist`` 136, ``rbf`` 159, ``manhattan`` 186, ``_dist`` 209 with symmetric /
full ring pipelines 265-486).

Split rules are the reference's: X split 0 -> result split 0; X replicated and Y split 0 ->
result split 1; both replicated -> replicated. The local tiles are produced by the native CDNA4
kernels (``ops.cdist``): the L2 family by the quadratic expansion on the FP16 matrix cores as a
3-term fp16 split with fp32 accumulation (``cdist_f16x3.hip``, fp32-GEMM accuracy; the exact
difference kernel for ``quadratic_expansion=False``) with a fused clamp / sqrt / exp epilogue, L1
on the VALU. When both operands are split, Y's blocks are either all-gathered once (fits in
memory) or streamed around a double-buffered ring (``HEAT_RING_MODE=direct``: posted to all peers
at once) that overlaps each transfer with the previous tile's kernel.
"""
from __future__ import annotations

from typing import Callable, Optional

import torch

from ..core import types
from ..core.dndarray import DNDarray
from ..core.communication import MPI
from .. import ops
from ..parallel.ring import ring_pass

__all__ = ["cdist", "cdist_stream", "manhattan", "rbf"]

_ALLGATHER_BYTES = 2 << 30


# local metrics (torch tensors) --------------------------------------------------------------
def _euclidian(x: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
    return ops.cdist(x, y, "euclidean")


def _euclidian_fast(x: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
    return ops.cdist(x, y, "euclidean")


def _quadratic_expand(x: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
    return ops.cdist(x, y, "sqeuclidean")


def _gaussian(x: torch.Tensor, y: torch.Tensor, sigma: float = 1.0) -> torch.Tensor:
    return ops.cdist(x, y, "gaussian", sigma=sigma)


_gaussian_fast = _gaussian


def _manhattan(x: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
    return ops.cdist(x, y, "manhattan")


_manhattan_fast = _manhattan


def cdist(X: DNDarray, Y: Optional[DNDarray] = None, quadratic_expansion: bool = False) -> DNDarray:
    """Euclidean distance matrix ``d(x, y) = sqrt(|x - y|^2)`` of size m x n.

    ``quadratic_expansion=True``: |x|^2 + |y|^2 - 2 x.y with the x.y GEMM as a 3-term fp16 split on
    the FP16 matrix cores (``cdist_f16x3.hip``, fp32-GEMM accuracy; fp64 input uses fp64 math),
    fastest; like any expansion it cancels to ~sqrt(eps |x|^2) for near-identical rows.
    ``False``: exact difference-based kernel (no cancellation for near-identical rows)."""
    return _dist(X, Y, "euclidean", exact=not quadratic_expansion)


def rbf(X: DNDarray, Y: Optional[DNDarray] = None, sigma: float = 1.0, quadratic_expansion: bool = False) -> DNDarray:
    """Gaussian kernel matrix ``exp(-|x - y|^2 / (2 sigma^2))``."""
    return _dist(X, Y, "gaussian", sigma, exact=not quadratic_expansion)


def manhattan(X: DNDarray, Y: Optional[DNDarray] = None, expand: bool = False) -> DNDarray:
    """Manhattan (L1) distance matrix."""
    return _dist(X, Y, "manhattan")


def _dist(X: DNDarray, Y: Optional[DNDarray] = None, metric="euclidean", sigma: float = 1.0,
          exact: bool = True) -> DNDarray:
    """Pairwise ``metric`` between rows of X and Y (Y = X if None)."""
    if callable(metric):
        return _dist_callable(X, Y, metric)

    def _local(metric, x, y, sigma, out=None):
        return ops.cdist(x, y, metric, sigma=sigma, out=out, exact=exact)

    if not isinstance(X, DNDarray):
        raise TypeError("X must be a DNDarray")
    if len(X.shape) > 2:
        raise NotImplementedError("Only 2D data matrices are currently supported")
    if Y is None:
        Y = X
    if not isinstance(Y, DNDarray):
        raise TypeError("Y must be a DNDarray or None")
    if len(Y.shape) > 2:
        raise NotImplementedError("Only 2D data matrices are currently supported")
    if X.gshape[1] != Y.gshape[1]:
        raise ValueError("X and Y must have the same number of features, got {} and {}".format(X.gshape[1], Y.gshape[1]))
    if X.split not in (None, 0) or Y.split not in (None, 0):
        raise NotImplementedError("Splittings other than 0 or None currently not supported.")
    dtype = types.promote_types(types.promote_types(X.dtype, Y.dtype), types.float32)
    if dtype not in (types.float32, types.float64):
        raise NotImplementedError("Datatype {} currently not supported as input".format(dtype))
    tt = dtype.torch_type()
    x = X.larray.to(tt)
    y = Y.larray.to(tt)
    m, n = X.gshape[0], Y.gshape[0]
    comm = X.comm
    dx, dy = X.is_distributed(), Y.is_distributed()
    if not dx and not dy:
        # the split rules hold in a world of one too
        out_split = 0 if X.split == 0 else (1 if Y.split == 0 else None)
        return DNDarray(_local(metric, x, y, sigma).to(tt), (m, n), dtype, out_split, X.device, comm, True)
    if dx and not dy:
        return DNDarray(_local(metric, x, y, sigma).to(tt), (m, n), dtype, 0, X.device, comm, X.balanced)
    if not dx and dy:
        return DNDarray(_local(metric, x, y, sigma).to(tt), (m, n), dtype, 1, X.device, comm, Y.balanced)
    counts, displs = Y.counts_displs()
    ybytes = n * Y.gshape[1] * y.element_size()
    if ybytes <= _ALLGATHER_BYTES:
        yfull = comm.allgather_tensor(y.contiguous(), 0, counts)
        res = _local(metric, x, yfull, sigma).to(tt)
        return DNDarray(res, (m, n), dtype, 0, X.device, comm, X.balanced)
    out = torch.empty((x.shape[0], n), dtype=tt, device=x.device)

    def tile(block: torch.Tensor, src: int):
        c0, cn = displs[src], counts[src]
        if cn and x.shape[0]:
            if tt == torch.float32 and out.is_cuda:
                _local(metric, x, block, sigma, out=out[:, c0: c0 + cn])
            else:
                out[:, c0: c0 + cn] = _local(metric, x, block, sigma)

    ring_pass(y, tile, comm, counts)
    return DNDarray(out, (m, n), dtype, 0, X.device, comm, X.balanced)


def _dist_callable(X: DNDarray, Y: Optional[DNDarray], fn: Callable) -> DNDarray:
    """User-supplied torch metric ``fn(x_block, y_block) -> tile`` (reference API)."""
    if Y is None:
        Y = X
    dtype = types.promote_types(types.promote_types(X.dtype, Y.dtype), types.float32)
    tt = dtype.torch_type()
    x, y = X.larray.to(tt), Y.larray.to(tt)
    m, n = X.gshape[0], Y.gshape[0]
    if X.is_distributed() and Y.is_distributed():
        y = X.comm.allgather_tensor(y.contiguous(), 0, Y.split_counts())
        split = 0
    elif X.is_distributed():
        split = 0
    elif Y.is_distributed():
        split = 1
    else:
        split = 0 if X.split == 0 else (1 if Y.split == 0 else None)
    return DNDarray(fn(x, y).to(tt), (m, n), dtype, split, X.device, X.comm, True)


def cdist_stream(X: DNDarray, Y: Optional[DNDarray], consume: Callable[[torch.Tensor, int, int], None],
                 metric: str = "euclidean", sigma: float = 1.0, tile: int = 65536,
                 quadratic_expansion: bool = True) -> None:
    """Distance matrix too large for memory (e.g. 1e6 x 1e6: 4 TB in fp32), produced tile by tile.

    For every (local row tile, global column tile) the native kernel writes the distances into
    ONE reused ``tile x tile`` device buffer and calls ``consume(d_tile, global_row0, global_col0)``
    (reduce it to kNN / row minima / a histogram / a threshold graph ...). ``Y`` blocks travel
    around the ring (``parallel.ring_pass``), overlapped with the tile compute. No extension in the
    reference, which materialises the whole matrix (``heat/spatial/distance.py:265-362``)."""
    if Y is None:
        Y = X
    if X.split not in (None, 0) or Y.split not in (None, 0):
        raise NotImplementedError("Splittings other than 0 or None currently not supported.")
    tile = max(128, tile // 128 * 128)  # packed operands are sliced at multiples of 128 rows
    x = X.larray if X.larray.dtype == torch.float32 else X.larray.float()
    y = Y.larray if Y.larray.dtype == torch.float32 else Y.larray.float()
    comm = X.comm
    r0 = X.counts_displs()[1][comm.rank] if X.is_distributed() else 0
    buf = torch.empty((min(tile, max(1, x.shape[0])), min(tile, max(1, Y.gshape[0]))), dtype=torch.float32,
                      device=x.device)
    exact = not quadratic_expansion
    # quadratic expansion on the device: pack X once (fp16x3 planes), each Y block once per visit
    packable = (not exact and metric != "manhattan" and x.is_cuda and ops.use_native(x))
    px = ops.cdist_pack(x) if packable and x.shape[0] else None

    def visit(block: torch.Tensor, c0: int):
        pb = ops.cdist_pack(block) if px is not None and block.shape[0] else None
        for i in range(0, x.shape[0], tile):
            xi = x[i: i + tile]
            for j in range(0, block.shape[0], tile):
                yj = block[j: j + tile]
                d = buf[: xi.shape[0], : yj.shape[0]]
                if pb is not None:
                    ops.cdist(xi, yj, metric, sigma=sigma, out=d, packed_x=px.rows(i, i + tile),
                              packed_y=pb.rows(j, j + tile))
                else:
                    ops.cdist(xi, yj, metric, sigma=sigma, out=d, exact=exact)
                consume(d, r0 + i, c0 + j)

    if Y.is_distributed():
        counts, displs = Y.counts_displs()
        ring_pass(y.contiguous(), lambda blk, src: visit(blk, displs[src]), comm, counts)
    else:
        visit(y, 0)
