"""Local GEMM / QR blocking below the BLAS operand limit (>4 GB device operands fault in
rocBLAS); exercised on CPU with a tiny limit."""
import importlib

import pytest
import torch

basics = importlib.import_module("heat_amd.core.linalg.basics")
qrmod = importlib.import_module("heat_amd.core.linalg.qr")


@pytest.fixture
def tiny_limit(monkeypatch):
    monkeypatch.setattr(basics, "_BLAS_MAX_BYTES", 64 * 1024)
    monkeypatch.setattr(basics, "_CHUNK_ON_HOST", True)


def test_mm_blocks(tiny_limit):
    g = torch.Generator().manual_seed(0)
    a = torch.randn(3000, 40, generator=g, dtype=torch.float64)
    b = torch.randn(40, 50, generator=g, dtype=torch.float64)
    w = torch.randn(40, 5000, generator=g, dtype=torch.float64)
    assert torch.allclose(basics._mm(a, b), a @ b)          # row blocks
    assert torch.allclose(basics._mm(a.T, a), a.T @ a)      # contraction blocks
    assert torch.allclose(basics._mm(b.T, w), b.T @ w)      # column blocks


@pytest.mark.parametrize("calc_q", [True, False])
def test_local_qr_blocks(tiny_limit, calc_q):
    a = torch.randn(3000, 40, generator=torch.Generator().manual_seed(1), dtype=torch.float64)
    q, r = qrmod._local_qr(a, calc_q)
    ref_r = torch.linalg.qr(a, mode="r")[1]
    assert torch.allclose(r.abs(), ref_r.abs(), atol=1e-10)
    if calc_q:
        assert torch.allclose(q @ r, a, atol=1e-10)
        assert torch.allclose(q.T @ q, torch.eye(40, dtype=torch.float64), atol=1e-10)


def test_distributed_matmul_qr_blocked(tiny_limit):
    import heat_amd as ht

    x = ht.random.randn(2000, 30, split=0, dtype=ht.float64)
    y = ht.random.randn(30, 20, dtype=ht.float64)
    assert ht.allclose(ht.matmul(x, y), ht.array(x.numpy() @ y.numpy()))
    q, r = ht.linalg.qr(x)
    assert ht.allclose(ht.matmul(q, r), x, atol=1e-10)


@pytest.mark.parametrize("cond", [1.0, 1e3, 1e6])
@pytest.mark.parametrize("calc_q", [True, False])
def test_cholqr_accuracy(cond, calc_q):
    """CholeskyQR2 (well conditioned) and the shifted CholeskyQR3 fallback (ill conditioned):
    Q orthogonal to fp32 accuracy, Q R = A, R upper triangular with a positive diagonal."""
    import heat_amd as ht

    g = torch.Generator().manual_seed(3)
    u, _ = torch.linalg.qr(torch.randn(4000, 50, generator=g, dtype=torch.float64))
    v, _ = torch.linalg.qr(torch.randn(50, 50, generator=g, dtype=torch.float64))
    s = torch.logspace(0, -torch.log10(torch.tensor(cond)).item(), 50, dtype=torch.float64)
    a = ((u * s) @ v.T).float()
    x = ht.array(a, split=0)
    q, r = ht.linalg.qr(x, calc_q=calc_q, mode="reduced")
    R = r.larray
    assert torch.allclose(R, torch.triu(R))
    assert torch.all(torch.diagonal(R) > 0)
    ref = torch.linalg.qr(a.double(), mode="r")[1]
    ref = ref * torch.sign(torch.diagonal(ref)).unsqueeze(1)
    assert torch.allclose(R.double(), ref, atol=1e-5 * float(s.max()), rtol=1e-3)
    if calc_q:
        Q = q.numpy()
        assert abs(Q.T @ Q - torch.eye(50).numpy()).max() < 1e-5
        assert abs(Q @ R.numpy() - a.numpy()).max() < 1e-5
