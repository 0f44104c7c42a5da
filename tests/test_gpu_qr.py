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


@pytest.mark.parametrize("m,n", [(5000, 100), (20000, 256), (777, 65), (300, 300), (4097, 33), (30000, 700),
                                 (40, 6), (1000, 32), (5000, 17)])
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
    # bit-reproducible: the panel sums are fixed-order trees (no float atomics)
    q2, r2 = ops.householder_qr(a.to(dev), 0, m, True)
    assert torch.equal(q2, q) and torch.equal(r2, r)
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


# ------------------------------------------------------------ fp64 factor kernels (csrc/linalg64.hip)
@pytest.mark.parametrize("n", [1, 63, 64, 65, 200, 1000, 4096])
def test_cholesky_upper_device(n):
    from heat_amd import ops

    dev = _dev()
    g = torch.Generator().manual_seed(n)
    a = torch.randn(n + 7, n, generator=g, dtype=torch.float64)
    G = (a.T @ a).to(dev)
    R, info = ops.cholesky_upper(G)
    assert int(info.item()) == 0
    assert torch.equal(R, torch.triu(R)) and bool((torch.diagonal(R) > 0).all())
    rel = ((R.T @ R - G).abs().max() / G.abs().max()).item()
    assert rel < 1e-13 * max(1, n // 64), rel
    ref = torch.linalg.cholesky(G.cpu(), upper=True)
    assert torch.allclose(R.cpu(), ref, rtol=1e-9, atol=1e-9 * ref.abs().max().item())


def test_cholesky_upper_reports_breakdown():
    from heat_amd import ops

    dev = _dev()
    G = torch.eye(300, dtype=torch.float64)
    G[150, 150] = -1.0
    _, info = ops.cholesky_upper(G.to(dev))
    assert int(info.item()) == 151


@pytest.mark.parametrize("n", [1, 64, 100, 129, 513, 1000, 4096])
def test_tri_inv_upper_device(n):
    from heat_amd import ops

    dev = _dev()
    g = torch.Generator().manual_seed(3 * n)
    # a well-conditioned triangle (the Cholesky factor of a Gram matrix, cond ~ 1e2); a random
    # triangle's condition number grows like 2^n and no inverse is accurate for it
    a = torch.randn(n + 50, n, generator=g, dtype=torch.float64)
    R = torch.linalg.cholesky(a.T @ a, upper=True).to(dev)
    X = ops.tri_inv_upper(R)
    assert torch.equal(X, torch.triu(X))
    err = (X @ R - torch.eye(n, dtype=torch.float64, device=dev)).abs().max().item()
    assert err < 1e-12 * max(1, n // 16), err


@pytest.mark.parametrize("m,k,n", [(64, 64, 64), (100, 37, 300), (1000, 64, 1000), (3, 5, 7)])
@pytest.mark.parametrize("layout", ["nn", "tn", "nt", "tt"])
def test_gemm64_layouts_upper(m, k, n, layout):
    from heat_amd import ops

    dev = _dev()
    g = torch.Generator().manual_seed(m + k + n)
    a = torch.randn(m, k, generator=g, dtype=torch.float64)
    b = torch.randn(k, n, generator=g, dtype=torch.float64)
    A = a if layout[0] == "n" else a.t().contiguous().t()
    B = b if layout[1] == "n" else b.t().contiguous().t()
    c0 = torch.randn(m, n, generator=g, dtype=torch.float64)
    c = c0.clone().to(dev)
    ops.gemm64(A.to(dev), B.to(dev), out=c, alpha=-2.0, beta=0.5)
    ref = 0.5 * c0 - 2.0 * (a @ b)
    assert torch.allclose(c.cpu(), ref, rtol=1e-12, atol=1e-12 * k)
    cu = c0.clone().to(dev)
    ops.gemm64(A.to(dev), B.to(dev), out=cu, upper=True)
    mask = torch.ones(m, n, dtype=torch.bool).triu()
    assert torch.allclose(cu.cpu(), torch.where(mask, a @ b, c0), rtol=1e-12, atol=1e-12 * k)


@pytest.mark.parametrize("precision", ["highest", "high"])
@pytest.mark.parametrize("m,n", [(100_000, 256), (20_000, 300), (4096, 64)])
def test_cholqr_native_path(m, n, precision):
    """Device fp32 CholeskyQR2 on the hand-written kernels (gemm_tiled + linalg64): orthogonal Q,
    Q R = A to fp32-GEMM accuracy, R upper with a non-negative diagonal."""
    import heat_amd as ht

    dev = _dev()
    old = torch.get_float32_matmul_precision()
    torch.set_float32_matmul_precision(precision)
    try:
        a = _ill(m, n, 50.0, m + n, torch.float32)
        x = ht.array(a.to(dev), split=None)
        q, r = ht.linalg.qr(x, mode="reduced")
        Q, R = q.larray.double(), r.larray.double()
        orth = (Q.T @ Q - torch.eye(n, dtype=torch.float64, device=dev)).abs().max().item()
        assert orth < 5e-6, orth   # fp32 CholeskyQR2 with the fp64-summed split-K Gram
        rec = (Q @ R - a.to(dev).double()).abs().max().item() / a.abs().max().item()
        assert rec < 1e-5, rec
        assert torch.equal(R, torch.triu(R)) and bool((torch.diagonal(R) >= 0).all())
    finally:
        torch.set_float32_matmul_precision(old)


# ------------------------------------------------- two-level Householder / fp64 V^T C / split-K Gram
@pytest.mark.parametrize("m,nc,N", [(100_000, 256, 1000), (5000, 256, 256), (777, 130, 333), (64, 3, 5),
                                    (300_001, 128, 128), (400_003, 32, 224), (70_000, 17, 300), (1000, 32, 31)])
@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
def test_vtc64(m, nc, N, dtype):
    """V^T C on the fp64 matrix cores: exact products, fp64 accumulation, against an fp64 GEMM
    (vector and scalar load variants, the narrow nc <= 32 kernel with its two-level split sum,
    row/column edges, split-K chunk tails)."""
    from heat_amd import ops

    dev = _dev()
    g = torch.Generator().manual_seed(m + nc + N)
    V = torch.randn(m, nc, generator=g, dtype=dtype).to(dev)
    C = torch.randn(m, N, generator=g, dtype=dtype).to(dev)
    W = ops.vtc64(V, C)
    ref = V.double().T @ C.double()
    scale = (V.double().abs().T @ C.double().abs()).max().item()
    assert (W - ref).abs().max().item() < 1e-13 * scale
    # column-offset views (unaligned base: the scalar-load kernel) and accumulation
    W2 = ops.vtc64(V[:, 1:], C[:, 1:], out=W[1:, 1:].contiguous(), accumulate=True)
    assert torch.allclose(W2, 2 * ref[1:, 1:], rtol=1e-12, atol=1e-12 * scale)
    # deterministic: bitwise equal on a re-run
    assert torch.equal(ops.vtc64(V, C), W)


@pytest.mark.parametrize("m,nc,N,group_bytes", [(300_001, 256, 1000, 1 << 30), (100_000, 256, 3840, 1 << 24),
                                               (5000, 64, 256, 1 << 30), (70_000, 36, 300, 1 << 30)])
def test_vtc_f32s(m, nc, N, group_bytes, monkeypatch):
    """The sliced fp32-MFMA V^T C of the Householder update: fp32 sums inside 1024-row slices,
    fp64 across them (partial-buffer groups, slice tails), against an fp64 GEMM; deterministic;
    the wide-reflector path of _vtc uses it."""
    from heat_amd import ops
    from heat_amd.ops import kernels as K

    monkeypatch.setattr(K, "_GRAM_PARTIAL_BYTES", group_bytes)
    dev = _dev()
    g = torch.Generator().manual_seed(m + nc + N)
    V = torch.randn(m, nc, generator=g).to(dev)
    C = torch.randn(m, N, generator=g).to(dev)
    W = K.vtc_f32s(V, C)
    assert W is not None and W.dtype == torch.float64
    ref = V.double().T @ C.double()
    bound = V.double().abs().T @ C.double().abs()
    rel = ((W - ref).abs() / bound).max().item()
    # one slice: fp32 accumulation of 1024 products (~u sqrt(1024) / 3 typical); the slices'
    # errors are independent, so the whole sum stays near that
    assert rel < 16 * 2.0 ** -24, rel
    assert torch.equal(K.vtc_f32s(V, C), W)
    assert torch.equal(K._vtc(V, C, True, None), W)


@pytest.mark.parametrize("exact", [True, False])
@pytest.mark.parametrize("m,n,group_bytes", [(200_000, 512, 1 << 30), (100_000, 300, 1 << 20), (9000, 256, 1 << 30),
                                              (50_000, 64, 1 << 16)])
def test_gram64_split_k(m, n, group_bytes, exact, monkeypatch):
    """Upper-triangle fp64 Gram from fp32 MFMA slices (several slice groups when the partial
    buffer is small): error at the fp32-per-slice level, far below a single fp32 sum."""
    from heat_amd import ops
    from heat_amd.ops import kernels as K

    dev = _dev()
    monkeypatch.setattr(K, "_GRAM_PARTIAL_BYTES", group_bytes)
    g = torch.Generator().manual_seed(m + n)
    x = (torch.randn(m, n, generator=g) * torch.logspace(0, 2, n)).to(dev)
    G = ops.gram64(x, exact=exact)
    ref = x.double().T @ x.double()
    up = torch.ones(n, n, dtype=torch.bool, device=dev).triu()
    assert torch.equal(G[~up], torch.zeros_like(G[~up]))
    d = torch.sqrt(torch.diagonal(ref))
    rel = ((G - ref).abs() / (d.unsqueeze(1) * d.unsqueeze(0)))[up].max().item()
    # fp32 accumulation inside a slice of kc rows, fp64 across slices: relative diagonal error
    # ~ u kc / (3 sqrt(m)) (one fp32 sum over all m rows: ~ u sqrt(m) / 3)
    kc = min(K._GRAM_KCHUNK, m)
    assert rel < 10 * 2.0 ** -24 * kc / m ** 0.5, rel


@pytest.mark.parametrize("precision", ["highest", "high"])
def test_householder_two_level_orthogonality_fp32(precision):
    """fp32 Householder with 256-column block reflectors (vtc64 + exact fp32 library update): Q is
    orthogonal to < 1e-6 for an ill-conditioned input, R matches the host algorithm - also when
    the caller set float32 matmul precision "high" (the update must not take the reduced-precision
    library path then)."""
    from heat_amd import ops

    dev = _dev()
    prev = torch.get_float32_matmul_precision()
    torch.set_float32_matmul_precision(precision)
    try:
        _householder_two_level_check(dev, ops)
    finally:
        torch.set_float32_matmul_precision(prev)
    assert torch.get_float32_matmul_precision() == prev


def _householder_two_level_check(dev, ops):
    a = _ill(60_000, 640, 1e8, 9, torch.float32)
    q, r = ops.householder_qr(a.to(dev), 0, a.shape[0], True)
    Q = q.double()
    orth = (Q.T @ Q - torch.eye(640, dtype=torch.float64, device=dev)).abs().max().item()
    assert orth < 1e-6, orth
    rec = (Q @ r.double() - a.to(dev).double()).abs().max().item() / a.abs().max().item()
    assert rec < 1e-5, rec


@pytest.mark.parametrize("rows,cols", [(1, 1), (4096, 4096), (300, 1000), (1000, 3)])
def test_gemv64_device(rows, cols):
    """fp64 matrix-vector product kernel (CholeskyQR2's condition estimate) against torch fp64,
    row-major and transposed-view inputs."""
    from heat_amd.ops import kernels as K

    dev = _dev()
    g = torch.Generator().manual_seed(rows + cols)
    m = torch.randn(rows, cols, generator=g, dtype=torch.float64).to(dev)
    x = torch.randn(cols, 1, generator=g, dtype=torch.float64).to(dev)
    y = K.gemv64(m, x)
    assert y.shape == (rows, 1)
    assert torch.allclose(y, m @ x, rtol=1e-12, atol=1e-12 * cols)
    yt = K.gemv64(m.T, torch.ones(rows, dtype=torch.float64, device=dev))
    assert torch.allclose(yt, m.sum(0), rtol=1e-12, atol=1e-12 * rows)
