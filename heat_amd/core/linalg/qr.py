"""
QR decomposition (reference ``heat/core/linalg/qr.py``: ``qr`` 17; split 0 tiled CAQR 314-846,
split 1 panel broadcast 849-1018).

MI355X design: tall-skinny input (every rank holds >= 2n rows) uses CholeskyQR2 / shifted
CholeskyQR3 on the matrix cores (``_cholqr``: Gram GEMM + one n x n all-reduce + fp64 Cholesky per
pass). When the Cholesky breaks down (cond(A) beyond ~6e7) the rows stay where they are and a
distributed blocked Householder QR runs instead (``ops.householder_qr``, csrc/householder.hip:
one kernel per panel column with an fp64 2-vector all-reduce, compact-WY trailing updates as
GEMMs with one all-reduce of V^T C per panel) - backward stable for any conditioning. Other
split-0 input uses TSQR - one local QR per rank, ONE all-gather of the p small R factors, a
redundant QR of the stacked R on every rank (no tree latency: p <= 8 per node) and one local
GEMM ``Q_r @ Q2_r`` to form Q. The reference's binary merge tree with per-tile sends and string tags
(``qr.py:477-846``) disappears. Column-split input stays column-split (``_qr_split1``: Householder
panel factorisation by the owner, reflector broadcast, H_j^T applied by the later ranks).

Q mode: the reference returns a complete m x m Q. That is kept for matrices whose complete Q
fits comfortably in memory (``mode=None`` -> "complete" when m*m elements <= 2**28); beyond that
(e.g. the 1e7 x 4096 north-star case) the economy ("reduced") Q of shape m x n is returned.
"""
from __future__ import annotations

import os

import collections
from typing import Optional, Tuple, Union

import torch

from .. import factories, types
from ..dndarray import DNDarray, _chunk_counts

__all__ = ["qr"]

QR = collections.namedtuple("QR", "Q, R")


def _complete_ok(m: int) -> bool:
    return m * m <= (1 << 28)


def qr(a: DNDarray, tiles_per_proc: Union[int, torch.Tensor] = 1, calc_q: bool = True, overwrite_a: bool = False,
       mode: Optional[str] = None) -> QR:
    """QR factorisation ``a = Q R`` of a 2-D DNDarray; returns ``QR(Q, R)`` (``Q`` None if not
    ``calc_q``). ``tiles_per_proc`` is accepted for API compatibility (TSQR needs no tiling)."""
    if not isinstance(a, DNDarray):
        raise TypeError("'a' must be a DNDarray")
    if not isinstance(tiles_per_proc, (int, torch.Tensor)):
        raise TypeError("tiles_per_proc must be an int or a torch.Tensor, currently {}".format(type(tiles_per_proc)))
    if not isinstance(calc_q, bool):
        raise TypeError("calc_q must be a bool, currently {}".format(type(calc_q)))
    if not isinstance(overwrite_a, bool):
        raise TypeError("overwrite_a must be a bool, currently {}".format(type(overwrite_a)))
    if isinstance(tiles_per_proc, torch.Tensor) and tiles_per_proc.numel() != 1:
        raise ValueError("tiles_per_proc must be a single element torch.Tenor or int, currently has {} entries"
                         .format(tiles_per_proc.numel()))
    if a.ndim != 2:
        raise ValueError("Array 'a' must be 2 dimensional")
    m, n = a.gshape
    if mode is None:
        mode = "complete" if _complete_ok(m) else "reduced"
    if mode not in ("complete", "reduced"):
        raise ValueError("mode must be 'complete' or 'reduced'")
    dtype = a.dtype if types.heat_type_is_inexact(a.dtype) else types.float32
    tt = dtype.torch_type()

    if not a.is_distributed():
        t = a.larray.to(tt)
        res = _cholqr(t, a.comm, calc_q, False) if mode == "reduced" and t.shape[0] >= 2 * n else None
        if res is not None:
            q, r = res
        elif mode == "reduced" and t.is_cuda:
            from ... import ops

            q, r = ops.householder_qr(t, 0, t.shape[0], calc_q)  # csrc/householder.hip
        elif mode == "reduced":
            q, r = _local_qr(t, calc_q)
        else:
            q, r = torch.linalg.qr(t, mode=mode)
        # the same normalisation as every distributed path: diag(R) >= 0
        k = min(r.shape)
        d = torch.sign(torch.diagonal(r[:k, :k]))
        d = torch.where(d == 0, torch.ones_like(d), d)
        # in place, and only when a sign flips (CholeskyQR's R has a positive diagonal already):
        # the former cat-of-products form copied the m x n Q twice (~16 ms at 1.25e6 x 4096)
        if not bool((d == 1).all()):
            r = r.clone() if r._base is not None else r
            r[:k] *= d.unsqueeze(1)
            if q is not None:
                q = q.clone() if q._base is not None else q
                q[:, :k] *= d.unsqueeze(0)
        R = DNDarray(r, tuple(r.shape), dtype, a.split, a.device, a.comm, True)
        Q = DNDarray(q, tuple(q.shape), dtype, a.split, a.device, a.comm, True) if calc_q else None
        return QR(Q, R)

    if a.split == 1 and m >= n and (mode == "reduced" or m == n):
        return _qr_split1(a, dtype, calc_q)

    if mode == "complete":
        # complete Q (m x m): distributed Householder, Q's rows formed locally - no gather
        return _qr_complete(a, dtype, calc_q)

    src = a if a.split == 0 else _resplit(a, 0)
    if not src.is_balanced():
        src = src.copy()
        src.balance_()
    Ql, R2 = _tsqr(src.larray.to(tt), src.comm, n, calc_q)
    k = min(m, n)
    if mode == "complete" and m > R2.shape[0]:
        R2 = torch.cat([R2, R2.new_zeros((m - R2.shape[0], n))], dim=0)
    R = factories.array(R2, split=a.split, device=a.device, comm=a.comm, dtype=dtype)
    if not calc_q:
        return QR(None, R)
    Q = DNDarray(Ql, (m, k), dtype, 0, a.device, a.comm, True)
    if a.split == 1:
        Q = _resplit(Q, 1)
    return QR(Q, R)


def _qr_split1(a: DNDarray, dtype, calc_q: bool):
    """Column-split QR without redistributing rows (reference ``qr.py:849-1018``, panel
    broadcast): rank j, in column order, factors rows [c_j, m) of its (already updated) column
    panel with the blocked Householder kernels (``ops.householder_factor``) and broadcasts the
    reflectors + compact-WY T blocks; every later rank applies H_j^T to its own panel. Q is then
    accumulated backwards (Q_k = H_0 ... H_k E_k) with a second broadcast of each rank's
    reflectors. Backward stable for any conditioning; Q and R come out split along axis 1 with the
    input's column partition; memory O(local + 1 panel)."""
    from ... import ops

    comm = a.comm
    tt = dtype.torch_type()
    m, n = a.gshape
    counts, displs = a.counts_displs()
    me, p = comm.rank, comm.size
    dev = a.larray.device
    A = a.larray.to(tt).contiguous().clone()
    nb = ops.householder_block(A)
    mine = None      # (reflectors, panels) of this rank's column panel
    signs = {}       # sign(diag R_jj) of every panel j <= me

    def panel_shapes(j):
        rows, nj = m - displs[j], counts[j]
        return (rows, nj), [(k0, min(nb, nj - k0)) for k0 in range(0, nj, nb)]

    def send(j, fact):
        """Broadcast panel j's reflectors and T blocks from rank j; returns them on every rank."""
        shape, blocks = panel_shapes(j)
        if j == me:
            V, panels = fact
            T = torch.zeros((len(blocks), nb, nb), dtype=torch.float64, device=dev)
            for i, (_, nc, Tm) in enumerate(panels):
                T[i, :nc, :nc] = Tm
        else:
            V = torch.empty(shape, dtype=tt, device=dev)
            T = torch.empty((len(blocks), nb, nb), dtype=torch.float64, device=dev)
        comm.Bcast(V, root=j)
        comm.Bcast(T, root=j)
        return V, [(k0, nc, T[i, :nc, :nc]) for i, (k0, nc) in enumerate(blocks)]

    def diag_signs(V, nj):
        d = torch.sign(torch.diagonal(V[:nj, :nj]))
        return torch.where(d == 0, torch.ones_like(d), d)

    last = max((j for j in range(p) if counts[j]), default=-1)
    for j in range(p):
        nj = counts[j]
        if nj == 0:
            continue
        fact = None
        if j == me:
            fact = ops.householder_factor(A[displs[j]:], 0, m - displs[j])
            mine = fact
            A[displs[j]:] = fact[0]
        if j == last:
            if j == me:
                signs[j] = diag_signs(fact[0], nj)
            break
        V, panels = send(j, fact)
        signs[j] = diag_signs(V, nj)
        if me > j and counts[me]:
            ops.householder_apply(V, panels, A[displs[j]:], 0, transpose=True)

    # R: rows of panel j (< me) were produced by H_j^T, this rank's diagonal block is triu(V)
    nloc = counts[me]
    R = A.new_zeros((n, nloc))
    if nloc:
        top = displs[me]
        R[:top] = A[:top]
        R[top: top + nloc] = torch.triu(A[top: top + nloc])
        for j, d in signs.items():
            R[displs[j]: displs[j] + counts[j]] *= d.unsqueeze(1)
    Rd = DNDarray(R, (n, n), dtype, 1, a.device, comm, a.balanced)
    if not calc_q:
        return QR(None, Rd)
    # Q_k = H_0 H_1 ... H_k [0; I; 0]: own reflectors first, then every earlier panel's, in
    # descending order (panel j's reflectors are broadcast a second time)
    Q = A.new_zeros((m, nloc))
    if nloc:
        Q[displs[me]: displs[me] + nloc] = torch.eye(nloc, dtype=tt, device=dev)
    for j in range(last, -1, -1):
        if counts[j] == 0:
            continue
        if j == me:
            ops.householder_apply(mine[0], mine[1], Q[displs[j]:], 0, transpose=False, identity_start=True)
        if any(counts[k] for k in range(j + 1, p)):
            V, panels = send(j, mine if j == me else None)
            if me > j and nloc:
                ops.householder_apply(V, panels, Q[displs[j]:], 0, transpose=False)
    if nloc:
        Q *= signs[me].unsqueeze(0)
    return QR(DNDarray(Q, (m, n), dtype, 1, a.device, comm, a.balanced), Rd)


def _qr_complete(a: DNDarray, dtype, calc_q: bool) -> QR:
    """Complete QR (Q m x m) of a distributed matrix without gathering it.

    m >= n: the rows are distributed (a column-split input is redistributed once), blocked
    Householder with one fp64 all-reduce per column / two per panel (``ops.householder_factor``),
    R (n x n) assembled by one all-reduce, and every rank forms ITS rows of the complete Q by
    applying the reflectors to its rows of the identity (``ops.householder_apply``: per panel one
    nb x m all-reduce). m < n: QR of the leading m x m block, then R = Q^T A as one distributed
    matmul. Q comes back split 0 (split 1 for a column-split input), R split like the input."""
    from ... import ops
    from ..communication import MPI
    from .basics import matmul, transpose, triu

    m, n = a.gshape
    comm = a.comm
    if m < n:
        lead = _resplit(a[:, :m], 0)
        q, _ = _qr_complete(lead, dtype, True)
        r = triu(matmul(transpose(q), a.astype(dtype)))
        r = r if r.split == a.split else _resplit(r, a.split)
        if calc_q and a.split == 1:
            q = _resplit(q, 1)
        return QR(q if calc_q else None, r)
    src = a if a.split == 0 else _resplit(a, 0)
    if not src.is_balanced():
        src = src.copy()
        src.balance_()
    tt = dtype.torch_type()
    local = src.larray.to(tt)
    counts = comm.allgather_sizes(local.shape[0])
    g0 = sum(counts[: comm.rank])

    def red(t):
        comm.Allreduce(MPI.IN_PLACE, t, MPI.SUM)
        return t

    A, panels = ops.householder_factor(local, g0, m, red)
    kmax = min(m, n)
    m_r = local.shape[0]
    R = torch.zeros((kmax, n), dtype=tt, device=local.device)
    lo, hi = max(g0, 0), min(g0 + m_r, kmax)
    if hi > lo:
        R[lo:hi] = torch.triu(A[lo - g0: hi - g0], diagonal=lo)
    red(R)
    d = torch.sign(torch.diagonal(R))
    d = torch.where(d == 0, torch.ones_like(d), d)
    R = d.unsqueeze(1) * R
    # R is m x n with zero rows past kmax: build only this rank's block of it (a replicated
    # m x n tensor would be as large as the whole input on every rank)
    off, lshape, _ = comm.chunk((m, n), a.split)
    Rl = R.new_zeros(lshape)
    if a.split == 1:
        Rl[:kmax] = R[:, off: off + lshape[1]]
    else:
        lo, hi = off, min(off + lshape[0], kmax)
        if hi > lo:
            Rl[: hi - lo] = R[lo:hi]
    Rd = DNDarray(Rl, (m, n), dtype, a.split, a.device, comm, True)
    if not calc_q:
        return QR(None, Rd)
    Q = torch.zeros((m_r, m), dtype=tt, device=local.device)
    if m_r:
        Q[torch.arange(m_r, device=Q.device), torch.arange(g0, g0 + m_r, device=Q.device)] = 1
    ops.householder_apply(A, panels, Q, g0, transpose=False, allreduce=red)
    Q[:, :kmax] *= d.unsqueeze(0)
    Qd = DNDarray(Q, (m, m), dtype, 0, a.device, comm, True)
    if a.split == 1:
        Qd = _resplit(Qd, 1)
    return QR(Qd, Rd)


def _resplit(x: DNDarray, axis):
    from ..manipulations import resplit

    return resplit(x, axis)


def _cholqr(local: torch.Tensor, comm, calc_q: bool, distributed: bool):
    """Tall-skinny QR by CholeskyQR2 on matrix-core GEMMs (Yamamoto et al. / Fukaya et al.).
    Per pass: Gram matrix G = A^T A (local GEMM at BLAS speed + ONE n x n all-reduce),
    R = chol(G) in fp64, Q = A R^{-1} as a GEMM with the explicit triangular inverse; two passes
    give an orthogonal Q for cond(A) up to ~1/sqrt(eps). The first attempt runs the GEMMs in the
    input precision; if a Cholesky breaks down (cond(A) beyond ~3e3 for fp32 input) the first pass
    is redone with fp64 GEMMs (good to cond(A) ~ 6e7). Returns (local Q rows or None, R), or None
    when neither applies (the caller falls back to Householder TSQR).

    rocSOLVER's Householder geqrf runs the 1.25e6 x 4096 per-GPU block at ~1 TFLOP/s; the GEMMs
    here run at ~150 TFLOP/s (fp32) / ~75 (fp64) (``benchmarks/linalg``)."""
    for precise in (False, True):
        res = _cholqr_attempt(local, comm, calc_q, distributed, precise)
        if res is not None:
            return res
    return None


# HEAT_QR_TRI=0: the R^-1 products as full GEMMs (A/B of the triangular-aware kernels)
_QR_TRI = os.environ.get("HEAT_QR_TRI", "1") != "0"


def _cholqr_native(A: torch.Tensor, comm, calc_q: bool, distributed: bool):
    """CholeskyQR2 of a device fp32 block entirely on the hand-written kernels: the Gram matrices
    (``ops.gram64``: upper-triangle tiles, split-K slices summed in fp64 - an fp64 Gram from fp32
    MFMA work) and both Q products on the 256-tile MFMA GEMMs (``ops/csrc/gemm_tiled.hip``, exact
    f32 or fused fp16x3 by the float32 matmul precision), the fp64 Cholesky and triangular inverse on
    ``ops/csrc/linalg64.hip`` (no rocSOLVER / rocBLAS). One n x n all-reduce per pass; one host
    sync per pass for the breakdown / conditioning decision."""
    from ... import ops
    from .basics import fgemm

    dt = A.dtype

    def allreduce(g: torch.Tensor) -> torch.Tensor:
        if distributed:
            from ..communication import MPI

            comm.Allreduce(MPI.IN_PLACE, g, MPI.SUM)
        return g

    def factor(G: torch.Tensor, first: bool):
        R, info = ops.cholesky_upper(G.double())
        Rinv = ops.tri_inv_upper(R)
        ok = int(info.item()) == 0 and bool(torch.isfinite(Rinv).all())
        if ok and first:
            ok = _cond_estimate_inv(R, Rinv) <= 1e3  # CholeskyQR2 with an fp32 Gram: cond(A) <~ 1e3
        if distributed:
            ok = comm.allreduce(int(ok)) == comm.size
        return (R, Rinv) if ok else (None, None)

    R1, Ri1 = factor(allreduce(ops.gram64(A)), True)
    if R1 is None:
        return None
    # R^-1 is upper triangular: output column tile n0 contracts only k < n0 + 256 (half the work)
    Q1 = fgemm(A, Ri1.to(dt), b_upper=_QR_TRI)
    R2, Ri2 = factor(allreduce(ops.gram64(Q1)), False)
    if R2 is None:
        return None
    R = ops.gemm64(R2, R1).to(dt)
    if not calc_q:
        return None, R
    Q = fgemm(Q1, Ri2.to(dt), b_upper=_QR_TRI)
    return Q, R


def _cond_estimate_inv(R: torch.Tensor, Rinv: torch.Tensor, iters: int = 12) -> float:
    """2-norm condition number estimate ||R|| ||R^-1|| by power iteration on R^T R and
    R^-T R^-1 (fp64 matrix-vector products on ``ops.gemv64``, the transposes copied once;
    deterministic start vector)."""
    from ...ops import kernels as _k

    n = R.shape[0]
    if n == 0:
        return 1.0
    g = torch.Generator(device="cpu").manual_seed(12345)
    x0 = (torch.rand(n, 1, generator=g, dtype=torch.float64) + 0.5).to(R.device)
    res = []
    for M in (R, Rinv):
        Mt = M.T.contiguous()
        x = x0 / x0.norm()
        s = 0.0
        for _ in range(iters):
            y = _k.gemv64(Mt, _k.gemv64(M, x))
            s = float(y.norm())
            if not 0.0 < s < float("inf"):
                return float("inf")
            x = y / s
        res.append(s)
    return (res[0] * res[1]) ** 0.5


def _cholqr_attempt(local: torch.Tensor, comm, calc_q: bool, distributed: bool, precise: bool):
    from .basics import _mm, _native_fp32

    if not precise and _native_fp32(local, local):
        return _cholqr_native(local, comm, calc_q, distributed)

    m_r, n = local.shape
    dt = local.dtype
    wide = torch.float64 if precise else dt
    step = max(1, (1 << 27) // max(n, 1))  # row blocks of transient products

    def allreduce(g: torch.Tensor) -> torch.Tensor:
        if distributed:
            from ..communication import MPI

            comm.Allreduce(MPI.IN_PLACE, g, MPI.SUM)
        return g

    # CholeskyQR2 is stable while cond(A) <~ u^{-1/2} of the Gram precision: a Cholesky that
    # "succeeds" beyond that returns an R whose Q has lost orthogonality (no breakdown to catch).
    # cond(R) = cond(A) is estimated by power / inverse iteration on R^T R (O(n^2) per step); past
    # the limit the caller goes on to the precise pass, then to Householder.
    cond_limit = 1e7 if wide == torch.float64 else 1e3

    def chol(g: torch.Tensor, first: bool = False):
        r, info = torch.linalg.cholesky_ex(g.double(), upper=True)
        ok = int(info) == 0 and bool(torch.isfinite(r).all())
        if ok and first:
            ok = _cond_estimate(r) <= cond_limit
        if distributed:
            ok = comm.allreduce(int(ok)) == comm.size
        return r if ok else None

    def tri_inv(r: torch.Tensor, to) -> torch.Tensor:
        eye = torch.eye(n, dtype=r.dtype, device=r.device)
        return torch.linalg.solve_triangular(r, eye, upper=True).to(to)

    def blocks(t: torch.Tensor):
        for r0 in range(0, t.shape[0], step):
            yield r0, t[r0: r0 + step]

    # pass 1 (in `wide` precision)
    g = local.new_zeros((n, n), dtype=wide)
    for _, blk in blocks(local):
        bw = blk.to(wide)
        g += _mm(bw.T, bw)
    r1 = chol(allreduce(g), first=True)
    if r1 is None:
        return None
    rinv = tri_inv(r1, wide)
    # pass 2: Q1 = A R1^{-1} (stored in the input precision), G2 = Q1^T Q1
    need_q = calc_q
    q = torch.empty_like(local) if need_q else None
    g = local.new_zeros((n, n))
    for r0, blk in blocks(local):
        qb = _mm(blk.to(wide), rinv).to(dt)
        if need_q:
            q[r0: r0 + qb.shape[0]] = qb
        g += _mm(qb.T, qb)
    r2 = chol(allreduce(g))
    if r2 is None:
        return None
    rtot = (r2 @ r1).to(dt)
    if not calc_q:
        return None, rtot
    rinv2 = tri_inv(r2, dt)
    for r0, blk in blocks(q):
        q[r0: r0 + blk.shape[0]] = _mm(blk, rinv2)
    return q, rtot


def _cond_estimate(r: torch.Tensor, iters: int = 12) -> float:
    """2-norm condition number estimate of an upper triangular R: power iteration on R^T R for the
    largest singular value, inverse iteration (two triangular solves per step) for the smallest.
    Deterministic start vector (every rank computes the same replicated R and the same answer)."""
    n = r.shape[0]
    if n == 0:
        return 1.0
    r = r.double()
    g = torch.Generator(device="cpu").manual_seed(12345)
    x0 = torch.rand(n, 1, generator=g, dtype=torch.float64).to(r.device) + 0.5
    x = x0 / x0.norm()
    smax = 0.0
    for _ in range(iters):
        y = r.T @ (r @ x)
        smax = float(y.norm())
        if smax == 0.0:
            return float("inf")
        x = y / smax
    x = x0 / x0.norm()
    inv = 0.0
    for _ in range(iters):
        z = torch.linalg.solve_triangular(r.T, x, upper=False)
        y = torch.linalg.solve_triangular(r, z, upper=True)
        inv = float(y.norm())
        if not inv < float("inf"):
            return float("inf")
        x = y / inv
    return (smax * inv) ** 0.5


def _local_qr(t: torch.Tensor, calc_q: bool = True):
    """Reduced QR of one rank's block. Device blocks above the BLAS operand limit (see
    ``basics._BLAS_MAX_BYTES``) are factorised as a local TSQR over row chunks: QR per chunk,
    QR of the stacked R factors, Q chunk = Q_i @ Q2_i."""
    from . import basics
    from .basics import _mm

    _BLAS_MAX_BYTES = basics._BLAS_MAX_BYTES
    m, n = t.shape
    if not (t.is_cuda or basics._CHUNK_ON_HOST) or t.numel() * t.element_size() <= _BLAS_MAX_BYTES or m <= 2 * n:
        if calc_q:
            return torch.linalg.qr(t, mode="reduced")
        return None, torch.linalg.qr(t, mode="r")[1]
    step = max(n, _BLAS_MAX_BYTES // (n * t.element_size()))
    qs, rs = [], []
    for r0 in range(0, m, step):
        blk = t[r0: r0 + step]
        if calc_q:
            q, r = torch.linalg.qr(blk, mode="reduced")
            qs.append(q)
        else:
            r = torch.linalg.qr(blk, mode="r")[1]
        rs.append(r)
    stacked = torch.cat(rs, 0)
    q2, r = torch.linalg.qr(stacked, mode="reduced")
    if not calc_q:
        return None, r
    out = torch.empty((m, r.shape[0]), dtype=t.dtype, device=t.device)
    off, row = 0, 0
    for q in qs:
        kq = q.shape[1]
        out[row: row + q.shape[0]] = _mm(q, q2[off: off + kq])
        off += kq
        row += q.shape[0]
    return out, r


def _tsqr(local: torch.Tensor, comm, n: int, calc_q: bool):
    """One-level TSQR. Returns (this rank's rows of Q, replicated R)."""
    m_r = local.shape[0]
    if local.is_floating_point() and comm.allreduce(int(m_r >= 2 * n)) == comm.size:
        res = _cholqr(local, comm, calc_q, True)
        if res is not None:
            return res
    if local.is_floating_point():
        # cond(A) beyond CholeskyQR's reach: distributed blocked Householder (one fp64 vector
        # all-reduce per column, two per panel; csrc/householder.hip) - backward stable for any
        # conditioning, Q orthogonal to working precision
        from ... import ops
        from ..communication import MPI

        counts = comm.allgather_sizes(m_r)
        g0 = sum(counts[: comm.rank])

        def red(t):
            comm.Allreduce(MPI.IN_PLACE, t, MPI.SUM)
            return t

        q, r = ops.householder_qr(local, g0, sum(counts), calc_q, red)
        return q, r
    if m_r > 0:
        q1, r1 = _local_qr(local, calc_q)  # q1: m_r x min(m_r,n), r1: min(m_r,n) x n
    else:
        q1 = local.new_zeros((0, 0))
        r1 = local.new_zeros((0, n))
    rows = comm.allgather_sizes(r1.shape[0])
    stacked = comm.allgather_tensor(r1.contiguous(), 0, rows)
    q2, r = torch.linalg.qr(stacked, mode="reduced")  # q2: sum(rows) x k
    # fix signs so that diag(R) >= 0 (deterministic, like LAPACK-normalised results)
    d = torch.sign(torch.diagonal(r))
    d = torch.where(d == 0, torch.ones_like(d), d)
    r = d.unsqueeze(1) * r
    q2 = q2 * d.unsqueeze(0)
    if not calc_q:
        return None, r
    off = sum(rows[: comm.rank])
    q2_r = q2[off: off + rows[comm.rank]]
    from .basics import _mm

    ql = _mm(q1, q2_r) if m_r > 0 else local.new_zeros((0, q2.shape[1]))
    return ql, r


DNDarray.qr = lambda self, tiles_per_proc=1, calc_q=True, overwrite_a=False: qr(self, tiles_per_proc, calc_q,
                                                                                 overwrite_a)
