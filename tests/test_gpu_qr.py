"""Blocked Householder QR kernels (``ops/csrc/householder.hip``) on the device against the host
reference path and fp64 checks; ill-conditioned inputs where CholeskyQR breaks down."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from heat_amd import ops

    assert ops.available(), "native library must load on a GPU box"
    return torch.device("cuda", 0)


def _ill(m, n, cond, seed, dtype):
    g = torch.Generator().manual_seed(seed)
    G = torch.randn(m, n, generator=g, dtype=torch.float64)
    V, _ = torch.linalg.qr(torch.randn(n, n, generator=g, dtype=torch.float64))
    s = torch.logspace(0, -torch.log10(torch.tensor(cond)).item(), n, dtype=torch.float64)
    return ((G * s) @ V.T).to(dtype)


@pytest.mark.parametrize("m,n", [(5000, 100), (20000, 256), (777, 65), (300, 300), (4097, 33)])
@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
def test_householder_qr_device(m, n, dtype):
    from heat_amd import ops

    dev = _dev()
    a = _ill(m, n, 1e10, m + n, dtype)
    q, r = ops.householder_qr(a.to(dev), 0, m, True)
    eps = torch.finfo(dtype).eps
    k = min(m, n)
    orth = (q.double().T @ q.double() - torch.eye(k, dtype=torch.float64, device=dev)).abs().max().item()
    assert orth < 200 * n * eps, orth
    rec = (q.double() @ r.double() - a.to(dev).double()).abs().max().item()
    assert rec < 200 * n * eps * a.abs().max().item(), rec
    assert torch.equal(r, torch.triu(r))
    assert torch.all(torch.diagonal(r) >= 0)
    # the host reference path of the same algorithm agrees
    qh, rh = ops.householder_qr(a, 0, m, True)
    assert torch.allclose(rh.double(), r.cpu().double(), rtol=1e3 * eps, atol=1e3 * eps * a.abs().max().item())


def test_ht_qr_ill_conditioned_uses_householder(gpu):
    import heat_amd as ht

    a = _ill(30000, 200, 1e10, 3, torch.float32)
    A = ht.array(a.numpy(), split=0)
    q, r = ht.linalg.qr(A, mode="reduced")
    qt = q.larray.double()
    assert (qt.T @ qt - torch.eye(200, dtype=torch.float64, device=qt.device)).abs().max().item() < 1e-5
    rec = (qt @ r.larray.double() - A.larray.double()).abs().max().item()
    assert rec < 1e-5 * A.larray.abs().max().item()
