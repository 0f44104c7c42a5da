"""Two-level blocked Householder QR (``ops.householder_factor``: 32-column panels inside outer
block reflectors with T = (striu(V^T V) + diag(1/tau))^-1) on the host path: orthogonality,
reconstruction and agreement with the one-level algorithm and LAPACK, for outer widths that do
and do not divide n, wide and tall inputs, fp32 (row blocks of a distributed matrix: the dist checks)."""
import pytest
import torch

from heat_amd import ops
from heat_amd.ops import kernels as K


def _qr(a, outer, monkeypatch):
    monkeypatch.setenv("HEAT_HH_OUTER", str(outer))
    return ops.householder_qr(a.clone(), 0, a.shape[0], True)


@pytest.mark.parametrize("m,n", [(300, 200), (257, 130), (96, 96), (50, 170)])
@pytest.mark.parametrize("outer", [32, 64, 96, 256])
def test_two_level_matches_lapack(m, n, outer, monkeypatch):
    g = torch.Generator().manual_seed(m * 7 + n)
    a = torch.randn(m, n, generator=g, dtype=torch.float64)
    q, r = _qr(a, outer, monkeypatch)
    k = min(m, n)
    assert q.shape == (m, k) and r.shape == (k, n)
    assert torch.allclose(q @ r, a, atol=1e-12 * n)
    assert torch.allclose(q.T @ q, torch.eye(k, dtype=torch.float64), atol=1e-13 * m)
    qr_, rr = torch.linalg.qr(a)
    d = torch.sign(torch.diagonal(rr))
    assert torch.allclose(r, d.unsqueeze(1) * rr, atol=1e-10)


def test_outer_block_T_is_the_larft_product(monkeypatch):
    """The block T from the UT identity equals the recursive-merge (LAPACK larft) T of the same
    reflectors: Q_b = I - V T V^T = H_1 ... H_k."""
    g = torch.Generator().manual_seed(3)
    a = torch.randn(200, 100, generator=g, dtype=torch.float64)
    monkeypatch.setenv("HEAT_HH_OUTER", "64")
    A, panels = ops.householder_factor(a.clone())
    assert [(k0, nc) for k0, nc, _ in panels] == [(0, 64), (64, 36)]
    rows = torch.arange(200).unsqueeze(1)
    for k0, nc, T in panels:
        V = K._hh_v(A, rows, k0, nc, 0)
        Qb = torch.eye(200, dtype=torch.float64) - V @ T @ V.T
        prod = torch.eye(200, dtype=torch.float64)
        for c in range(nc):
            v = V[:, c: c + 1]
            tau = 2.0 / float(v.T @ v)
            prod = prod @ (torch.eye(200, dtype=torch.float64) - tau * v @ v.T)
        assert torch.allclose(Qb, prod, atol=1e-12)
        assert torch.allclose(T, torch.triu(T))


def test_fp32_two_level(monkeypatch):
    """fp32 input: fp64-accumulated V^T C keeps the orthogonality at the fp32 rounding level."""
    monkeypatch.setenv("HEAT_HH_OUTER", "64")
    g = torch.Generator().manual_seed(11)
    a = torch.randn(400, 150, generator=g, dtype=torch.float32)
    q, r = ops.householder_qr(a.clone(), 0, 400, True)
    assert torch.allclose((q.double() @ r.double()), a.double(), atol=1e-4)
    err = (q.double().T @ q.double() - torch.eye(150, dtype=torch.float64)).abs().max()
    assert err < 5e-6
    qr_, rr = torch.linalg.qr(a.double())
    d = torch.sign(torch.diagonal(rr))
    assert torch.allclose(r.double(), d.unsqueeze(1) * rr, atol=1e-3)


def test_householder_block_width(monkeypatch):
    monkeypatch.setenv("HEAT_HH_OUTER", "96")
    assert ops.householder_block(torch.zeros(2, 2)) == 96
    monkeypatch.setenv("HEAT_HH_OUTER", "100")
    assert ops.householder_block(torch.zeros(2, 2)) == 96   # rounded down to the panel width
    monkeypatch.delenv("HEAT_HH_OUTER")
    assert ops.householder_block(torch.zeros(2, 2)) == 64


def test_vtc64_host_matches_fp64():
    g = torch.Generator().manual_seed(2)
    V = torch.randn(1000, 40, generator=g)
    C = torch.randn(1000, 70, generator=g)
    W = ops.vtc64(V, C)
    assert W.dtype == torch.float64
    assert torch.allclose(W, V.double().T @ C.double(), atol=1e-10)
    W2 = ops.vtc64(V, C, out=W.clone(), accumulate=True)
    assert torch.allclose(W2, 2 * W)
