"""Singular value decomposition (the reference ships an empty placeholder, ``linalg/svd.py``).

``svd`` here is a convenience: tall distributed matrices use TSQR + a small local SVD of R (U
stays split 0; a column-split input is redistributed to rows first), wide ones the same on the
transpose (V split 0). The matrix is never gathered; only the n x n factor R is replicated."""
from __future__ import annotations

import torch

from .. import factories, types
from ..dndarray import DNDarray

__all__ = ["svd"]


def svd(a: DNDarray, full_matrices: bool = False, compute_uv: bool = True):
    """Thin SVD. Split 0 (tall-skinny): ``A = QR`` (TSQR), ``R = U_r S V^T`` locally, ``U = Q U_r``."""
    from .qr import qr
    from .basics import matmul

    if a.ndim != 2:
        raise ValueError("svd requires a 2-D DNDarray")
    if full_matrices:
        raise NotImplementedError("full_matrices=True is not supported")
    if a.is_distributed() and a.gshape[1] > a.gshape[0]:
        # wide: A^T is tall (a local transpose; split 0 <-> 1), and A^T = U' S V'^T gives
        # A = V' S U'^T - no gather of A
        from .basics import transpose

        res = svd(transpose(a), full_matrices=False, compute_uv=compute_uv)
        if not compute_uv:
            return res
        u2, s2, v2 = res
        return v2, s2, u2
    if a.is_distributed():
        # tall: rows split (one redistribution when the columns were split), TSQR, a small local SVD
        # of R, U = Q U_r
        if a.split != 0:
            from ..manipulations import resplit

            a = resplit(a, 0)
        q, r = qr(a, mode="reduced")
        rt = r._gathered() if r.is_distributed() else r.larray
        ur, s, vh = torch.linalg.svd(rt, full_matrices=False)
        S = DNDarray(s, tuple(s.shape), types.canonical_heat_type(s.dtype), None, a.device, a.comm, True)
        if not compute_uv:
            return S
        U = matmul(q, factories.array(ur, device=a.device, comm=a.comm))
        V = DNDarray(vh.T.contiguous(), tuple(vh.T.shape), types.canonical_heat_type(vh.dtype), None, a.device,
                     a.comm, True)
        return U, S, V
    full = a._gathered() if a.is_distributed() else a.larray
    if not full.is_floating_point():
        full = full.float()
    u, s, vh = torch.linalg.svd(full, full_matrices=False)
    S = DNDarray(s, tuple(s.shape), types.canonical_heat_type(s.dtype), None, a.device, a.comm, True)
    if not compute_uv:
        return S
    U = factories.array(u, split=a.split, device=a.device, comm=a.comm) if a.split is not None else \
        DNDarray(u, tuple(u.shape), types.canonical_heat_type(u.dtype), None, a.device, a.comm, True)
    V = DNDarray(vh.T.contiguous(), tuple(vh.T.shape), types.canonical_heat_type(vh.dtype), None, a.device, a.comm, True)
    return U, S, V
