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

__all__ = ["cdist", "cdist_argmin", "cdist_stream", "cdist_topk", "manhattan", "rbf"]

_ALLGATHER_BYTES = 2 << 30
_SYM_MIN_F = 64   # compute-once symmetric tiles from this many features on (store-bound below)


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
        # the same block on both sides (Y = None on one rank, or a rank's diagonal block): the
        # difference kernels compute each distance pair once and mirror it - where that pays: they
        # write the distances at ~4 TB/s whatever they compute, and 2 f VALU ops per distance only
        # outweigh the 4-byte store from f ~ 64 (SUSY 40k x 18: 1.65 ms compute-once vs 1.59 ms
        # full, both store-bound; profiles/README.md round 5)
        return ops.cdist(x, y, metric, sigma=sigma, out=out, exact=exact,
                         symmetric=x is y and x.shape[-1] >= _SYM_MIN_F)

    if not isinstance(X, DNDarray):
        raise TypeError("X must be a DNDarray")
    if len(X.shape) > 2:
        raise NotImplementedError("Only 2D data matrices are currently supported")
    symmetric = Y is None
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
    y = x if symmetric else Y.larray.to(tt)
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
    if symmetric and ybytes > _allgather_bytes():
        # the half ring computes every off-diagonal tile pair once but RECEIVES half of the rank's
        # output over xGMI (~50-100x the time of writing it to HBM); below 2 GB of Y the
        # all-gather + local kernels win for every metric (see _local)
        out = torch.empty((x.shape[0], n), dtype=tt, device=x.device)
        _symmetric_half_ring(x, out, counts, displs, comm, lambda a, b: _local(metric, a, b, sigma).to(tt))
        return DNDarray(out, (m, n), dtype, 0, X.device, comm, X.balanced)
    if ybytes <= _allgather_bytes():
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


def _allgather_bytes() -> int:
    """Largest operand (bytes) that is all-gathered instead of streamed around the ring
    (``HEAT_CDIST_ALLGATHER_BYTES`` overrides, e.g. to exercise the ring paths in small tests)."""
    import os

    v = os.environ.get("HEAT_CDIST_ALLGATHER_BYTES")
    return int(v) if v else _ALLGATHER_BYTES


def _symmetric_half_ring(x: torch.Tensor, out: torch.Tensor, counts, displs, comm, tile) -> None:
    """``cdist(X)`` with X split 0 on p ranks: every off-diagonal tile pair computed ONCE (reference
    ``spatial/distance.py:237, 265-362``: d(X_r, X_q) = d(X_q, X_r)^T). Rank r computes its diagonal
    tile and the tiles (r, r - s) for s = 1 .. floor(p / 2) (for even p the pair r, r + p/2 is
    computed by the lower half only), and receives the mirrored tiles (r, r + s) from its partners.

    Overlap with bounded memory: the block exchange of step s + 1 is posted before tile s is
    computed, and each tile's transpose goes back (paired with the receive of the mirrored tile
    from r + s) while the next tile computes. At most two block exchanges and two tile exchanges
    are in flight: step s - 1's exchange is waited for, its mirrored tile copied into ``out`` and
    its buffers dropped right after step s is posted (the path runs when memory is the constraint,
    so holding every block or every transposed tile until the end is not an option). Every rank
    posts the same step sequence, so the point-to-point pairs match in order."""
    import torch.distributed as dist

    from ..parallel import staging as _SD

    p, r = comm.size, comm.rank
    rest = tuple(x.shape[1:])
    xs = x.contiguous()
    half = p // 2
    even = p % 2 == 0

    def computes(s_):  # does rank r compute the pair (r, r - s_)?
        return not (even and s_ == half) or r < half

    def post_block(s_):
        """Step s_'s block exchange: own block to r + s_, block of r - s_ in (-> (buffer, works))."""
        dst, src = (r + s_) % p, (r - s_) % p
        ops_, buf = [], None
        if computes(s_):
            buf = torch.empty((counts[src],) + rest, dtype=xs.dtype, device=xs.device)
            ops_.append(dist.P2POp(dist.irecv, buf, comm._g(src), comm.group))
        if not (even and s_ == half and r < half):
            ops_.insert(0, dist.P2POp(dist.isend, xs, comm._g(dst), comm.group))
        return buf, _SD.batch_isend_irecv(ops_)

    def finish(step):
        """Wait for a tile exchange, copy its mirrored tile into ``out``; its buffers die here."""
        works, dst, got, _tt = step
        for w in works:
            w.wait()
        if got is not None:
            out[:, displs[dst]: displs[dst] + counts[dst]] = got

    nxt = post_block(1) if half >= 1 else None
    out[:, displs[r]: displs[r] + counts[r]] = tile(xs, xs)    # overlaps the first block transfer
    prev = None
    for s_ in range(1, half + 1):
        dst, src = (r + s_) % p, (r - s_) % p
        block, works = nxt
        for w in works:
            w.wait()
        nxt = post_block(s_ + 1) if s_ < half else None      # lands under this step's tile
        tops, tt, got = [], None, None
        if computes(s_):
            t = tile(xs, block)
            del block
            out[:, displs[src]: displs[src] + counts[src]] = t
            tt = t.t().contiguous()
            del t
            tops.append(dist.P2POp(dist.isend, tt, comm._g(src), comm.group))
        if not (even and s_ == half and r < half):
            got = torch.empty((counts[r], counts[dst]), dtype=xs.dtype, device=xs.device)
            tops.append(dist.P2POp(dist.irecv, got, comm._g(dst), comm.group))
        cur = (_SD.batch_isend_irecv(tops), dst, got, tt)   # tt stays alive until its send is done
        if prev is not None:
            finish(prev)
        prev = cur
    if prev is not None:
        finish(prev)


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


def cdist_topk(X: DNDarray, Y: Optional[DNDarray] = None, k: int = 1):
    """The ``k`` nearest rows of ``Y`` (euclidean) for every row of ``X``, without the m x n
    distance matrix: ``(distances, indices)``, both (m, k), ascending, split like ``X``; the
    indices are global row numbers of ``Y``. Equal distances are ordered by index, so the result
    does not depend on the number of ranks (on the fused fp32 device kernel: among the candidates it
    returns - of exactly duplicated rows of ``Y`` at the k-th place it keeps one).

    The fused reduction the reference leaves to the caller (it materialises ``cdist`` and runs a
    distributed ``topk``, ``heat/classification/kneighborsclassifier.py:117-160``): device fp32 runs
    the fused MFMA distance + register top-k kernel (``ops.knn_topk``) per ``Y`` block, other inputs
    exact distance tiles in query blocks; a split ``Y`` circulates around the ring
    (``parallel.ring_pass``) and every rank keeps a running top-k of its own queries."""
    if Y is None:
        Y = X
    if not isinstance(X, DNDarray) or not isinstance(Y, DNDarray):
        raise TypeError("X and Y must be DNDarrays")
    if X.ndim != 2 or Y.ndim != 2:
        raise NotImplementedError("Only 2D data matrices are currently supported")
    if X.gshape[1] != Y.gshape[1]:
        raise ValueError("X and Y must have the same number of features, got {} and {}".format(X.gshape[1], Y.gshape[1]))
    if X.split not in (None, 0) or Y.split not in (None, 0):
        raise NotImplementedError("Splittings other than 0 or None currently not supported.")
    n = Y.gshape[0]
    if not isinstance(k, int) or k < 1 or k > n:
        raise ValueError("k must be an integer in [1, {}], got {}".format(n, k))
    dtype = types.promote_types(types.promote_types(X.dtype, Y.dtype), types.float32)
    if dtype not in (types.float32, types.float64):
        raise NotImplementedError("Datatype {} currently not supported as input".format(dtype))
    tt = dtype.torch_type()
    x = X.larray.to(tt)
    y = Y.larray.to(tt)
    nq = x.shape[0]
    best_d = torch.full((nq, k), float("inf"), dtype=tt, device=x.device)
    best_i = torch.full((nq, k), -1, dtype=torch.int64, device=x.device)

    def block_topk(block: torch.Tensor):
        kk = min(k, block.shape[0])
        if tt == torch.float32 and ops.use_native(x):
            dv, di = ops.knn_topk(x, block, kk)
            return dv.to(tt), di.to(torch.int64)
        step = max(1, (1 << 24) // max(block.shape[0], 1))  # <= 16M entries per tile (x3 tensors)
        ds, ids = [], []
        for q0 in range(0, nq, step):
            d = ops.cdist(x[q0: q0 + step], block, "sqeuclidean", exact=True).to(tt)
            # the kk smallest, ties at the kk-th value resolved to the lowest indices: everything
            # below the threshold, then the lowest-index entries equal to it
            thr = torch.topk(d, kk, dim=1, largest=False).values[:, -1:]
            col = torch.arange(d.shape[1], device=d.device).expand_as(d)
            key = torch.where(d < thr, torch.full_like(col, -1),
                              torch.where(d == thr, col, torch.full_like(col, d.shape[1])))
            di = torch.topk(key, kk, dim=1, largest=False).indices
            ds.append(torch.gather(d, 1, di))
            ids.append(di)
        return torch.cat(ds), torch.cat(ids)

    merged = [0]

    def merge(block: torch.Tensor, off: int):
        nonlocal best_d, best_i
        if block.shape[0] == 0 or nq == 0:
            return
        dv, di = block_topk(block)
        dv, di = dv.to(x.device), di.to(x.device) + off
        merged[0] += 1
        if merged[0] == 1 and dv.shape[1] == k and tt == torch.float32 and ops.use_native(x):
            # the first block's fused-kernel lists are already in (distance, index) order
            best_d, best_i = dv, di
            return
        cd = torch.cat([best_d, dv], dim=1)
        ci = torch.cat([best_i, di], dim=1)
        if tt == torch.float32:
            # one top-k over packed (distance bits, index) keys (distances are >= 0)
            best_d, best_i = ops.kernels._topk_lex(cd, ci, k, max_index=n - 1)
            return
        # (distance, index) order: stable sort by index, then stable sort by distance
        o = torch.sort(ci, dim=1, stable=True).indices
        cd, ci = torch.gather(cd, 1, o), torch.gather(ci, 1, o)
        o = torch.sort(cd, dim=1, stable=True).indices[:, :k]
        best_d, best_i = torch.gather(cd, 1, o), torch.gather(ci, 1, o)

    if Y.is_distributed():
        counts, displs = Y.counts_displs()
        ring_pass(y.contiguous(), lambda blk, src: merge(blk, displs[src]), Y.comm, counts)
    else:
        merge(y, 0)
    dist = torch.sqrt(torch.clamp(best_d, min=0))
    split = 0 if X.split == 0 else None
    bal = X.balanced if split is not None else True
    return (DNDarray(dist, (X.gshape[0], k), dtype, split, X.device, X.comm, bal),
            DNDarray(best_i, (X.gshape[0], k), types.int64, split, X.device, X.comm, bal))


def cdist_argmin(X: DNDarray, Y: Optional[DNDarray] = None):
    """Nearest row of ``Y`` for every row of ``X``: ``(distance, index)``, both (m,), split like
    ``X`` - :func:`cdist_topk` with k = 1 (vector quantisation / k-means ``predict`` without the
    distance matrix)."""
    d, i = cdist_topk(X, Y, 1)
    split = 0 if X.split == 0 else None
    bal = X.balanced if split is not None else True
    return (DNDarray(d.larray.reshape(-1), (X.gshape[0],), d.dtype, split, X.device, X.comm, bal),
            DNDarray(i.larray.reshape(-1), (X.gshape[0],), i.dtype, split, X.device, X.comm, bal))
