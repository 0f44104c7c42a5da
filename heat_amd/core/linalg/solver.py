"""
Iterative solvers (reference ``heat/core/linalg/solver.py``: ``cg`` 13, ``lanczos`` 68).

Lanczos re-orthogonalises against ALL previous Krylov vectors with one skinny GEMM and one GEMV
per step (``h = V^T w`` then ``w -= V h``) and TWO all-reduces per step in all (``[w.w, V^T w]``
before the matvec, ``[u.u, u^T A u]`` after it, the normalisation deferred past the matvec),
with no host synchronisation (the breakdown test selects on the device), instead of the
reference's two scalar all-reduces per (i, j) pair plus norms and dots (``solver.py:140-157``,
O(m^2) collectives).
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch

from .. import factories, types
from ..communication import MPI
from ..dndarray import DNDarray
from .basics import matmul, dot, norm

__all__ = ["cg", "lanczos"]


def cg(A: DNDarray, b: DNDarray, x0: DNDarray, out: Optional[DNDarray] = None) -> DNDarray:
    """Conjugate gradients for symmetric positive definite ``A x = b``."""
    if not isinstance(A, DNDarray) or not isinstance(b, DNDarray) or not isinstance(x0, DNDarray):
        raise TypeError("A, b and x0 need to be of type ht.DNDarray, but were {}, {}, {}".format(type(A), type(b),
                                                                                                  type(x0)))
    if A.ndim != 2:
        raise RuntimeError("A needs to be a 2D matrix")
    if b.ndim != 1:
        raise RuntimeError("b needs to be a 1D vector")
    if x0.ndim != 1:
        raise RuntimeError("c needs to be a 1D vector")
    r = b - matmul(A, x0)
    p = r
    rsold = matmul(r, r)
    x = x0
    for _ in range(len(b)):
        Ap = matmul(A, p)
        alpha = rsold / matmul(p, Ap)
        x = x + alpha * p
        r = r - alpha * Ap
        rsnew = matmul(r, r)
        if float(rsnew.item()) ** 0.5 < 1e-10:
            break
        p = r + (rsnew / rsold) * p
        rsold = rsnew
    if out is not None:
        out.larray = x.larray
        return out
    return x


def lanczos(A: DNDarray, m: int, v0: Optional[DNDarray] = None, V_out: Optional[DNDarray] = None,
            T_out: Optional[DNDarray] = None) -> Tuple[DNDarray, DNDarray]:
    """m Lanczos steps with full re-orthogonalisation: ``V`` (n x m, orthonormal), ``T`` (m x m tridiagonal)."""
    from .. import random as htrandom

    if not isinstance(A, DNDarray):
        raise TypeError("A needs to be of type ht.dndarra, but was {}".format(type(A)))
    if A.ndim != 2:
        raise RuntimeError("A needs to be a 2D matrix")
    if not isinstance(m, (int, float)):
        raise TypeError("m must be eiter int or float, but was {}".format(type(m)))
    m = int(m)
    n, column = A.shape
    if n != column:
        raise TypeError("Input Matrix A needs to be symmetric.")
    dtype = A.dtype if types.heat_type_is_inexact(A.dtype) else types.float32
    tt = dtype.torch_type()
    comm = A.comm
    vsplit = 0 if A.split == 0 else None
    if v0 is None:
        vr = htrandom.rand(n, split=vsplit, device=A.device, comm=comm)
        v0 = vr / norm(vr)
    else:
        if v0.split != vsplit:
            from ..manipulations import resplit

            v0 = resplit(v0, vsplit)
    dist = vsplit is not None and comm.is_distributed()
    dev = A.larray.device
    nloc = v0.lshape[0]
    V = torch.zeros((nloc, m), dtype=tt, device=dev)
    T = torch.zeros((m, m), dtype=tt, device=dev)

    def gdot(x: torch.Tensor) -> torch.Tensor:
        if dist:
            comm.Allreduce(MPI.IN_PLACE, x, MPI.SUM)
        return x

    def as_vec(t: torch.Tensor) -> DNDarray:
        return DNDarray(t, (n,), dtype, vsplit, A.device, comm, True)

    v = v0.larray.to(tt)
    w = matmul(A, as_vec(v)).larray.to(tt)
    alpha = gdot((w @ v).reshape(1))[0]
    w = w - alpha * v
    T[0, 0] = alpha
    V[:, 0] = v
    # breakdown replacements (beta ~ 0): drawn from a private generator so the global RNG state
    # does not depend on the step count, and selected on the device - no host sync per step
    # (one seed on every rank for replicated vectors, one per rank for their blocks)
    gen = torch.Generator(device=dev).manual_seed(0x5EED + (comm.rank if dist else 0))
    for i in range(1, m):
        # ONE all-reduce for beta^2 = w.w and the re-orthogonalisation coefficients of both the
        # residual w and its breakdown replacement r: [w.w, V^T w, V^T r] (V read once)
        r = torch.rand(w.shape, generator=gen, dtype=tt, device=dev)
        Vi = V[:, :i]
        red = torch.cat([(w @ w).reshape(1), (Vi.T @ torch.stack([w, r], 1)).T.reshape(-1)])
        red = gdot(red)
        beta = torch.sqrt(red[0])
        broke = beta < 1e-10
        h = torch.where(broke, red[1 + i:], red[1: 1 + i])
        u = torch.where(broke, r, w) - Vi @ h
        # normalisation deferred past the matvec: y = A u, then ONE all-reduce of [u.u, y.u] gives
        # |u| and alpha = u^T A u / u.u (the reference's dot after normalising, solver.py:140-157)
        y = matmul(A, as_vec(u)).larray.to(tt)
        red2 = gdot(torch.stack([u @ u, y @ u]))
        nrm = torch.sqrt(red2[0])
        vi = u / nrm
        alpha = red2[1] / red2[0]
        w = y / nrm - alpha * vi - beta * V[:, i - 1]
        T[i - 1, i] = beta
        T[i, i - 1] = beta
        T[i, i] = alpha
        V[:, i] = vi
    Vd = DNDarray(V, (n, m), dtype, vsplit, A.device, comm, True)
    if dist:
        Vd.resplit_(None)
    Td = DNDarray(T, (m, m), dtype, None, A.device, comm, True)
    if T_out is not None:
        T_out.larray = Td.larray.to(T_out.larray.dtype)
        Td = T_out
    if V_out is not None:
        V_out.larray = Vd.larray.to(V_out.larray.dtype)
        Vd = V_out
    return Vd, Td
