"""Exact fp32 MFMA GEMM (``ops/csrc/gemm_mfma.hip``) against an fp64 torch reference: every
operand layout, edge sizes (not multiples of the 128 x 128 x 16 tile), accumulate, row blocks."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from heat_amd import ops

    assert ops.available(), "native library must load on a GPU box"
    return torch.device("cuda", 0)


def _bound(a, b):
    # fp32 GEMM error bound class: ~K * 2^-24 * |a||b| elementwise (k-ordered fma chain)
    K = a.shape[1]
    return 4 * K * 2.0 ** -24 * (a.abs().double() @ b.abs().double()) + 1e-30


@pytest.mark.parametrize("m,k,n", [(300, 257, 129), (1024, 512, 768), (4099, 130, 65), (64, 4096, 64), (1, 7, 1),
                                   (129, 1, 131), (2000, 33, 3)])
@pytest.mark.parametrize("layout", ["nn", "tn", "nt", "tt"])
def test_gemm_f32_layouts(m, k, n, layout):
    from heat_amd import ops

    dev = _dev()
    g = torch.Generator().manual_seed(m * 7 + k * 3 + n)
    a = torch.randn(m, k, generator=g).to(dev)
    b = torch.randn(k, n, generator=g).to(dev)
    A = a if layout[0] == "n" else a.t().contiguous().t()
    B = b if layout[1] == "n" else b.t().contiguous().t()
    c = ops.gemm_f32(A, B)
    ref = a.double() @ b.double()
    assert torch.all((c.double() - ref).abs() <= _bound(a, b)), (c.double() - ref).abs().max()


def test_gemm_f32_accumulate_rowblock_and_gram():
    from heat_amd import ops

    dev = _dev()
    g = torch.Generator().manual_seed(5)
    x = torch.randn(3001, 70, generator=g).to(dev)
    gram = ops.gemm_f32(x.t(), x)                      # X^T X without a copy (k-major A)
    ref = x.double().t() @ x.double()
    assert torch.all((gram.double() - ref).abs() <= _bound(x.t(), x))
    out = torch.ones(500, 70, device=dev)
    big = torch.zeros(1000, 70, device=dev)
    ops.gemm_f32(x[:500], gram, out=out, accumulate=True)
    assert torch.allclose(out.double(), 1 + x[:500].double() @ gram.double(), rtol=1e-5, atol=1e-3)
    ops.gemm_f32(x[:300], gram, out=big[200:500])       # a row block of a larger result
    assert torch.allclose(big[200:500].double(), x[:300].double() @ gram.double(), rtol=1e-5, atol=1e-3)
    assert torch.all(big[:200] == 0) and torch.all(big[500:] == 0)


def test_gemm_f32_exact_products():
    """Integer-valued operands: every product and partial sum is exact in fp32, so the result must
    equal the integer matmul bit for bit (catches a transposed fragment map at once)."""
    from heat_amd import ops

    dev = _dev()
    g = torch.Generator().manual_seed(9)
    a = torch.randint(-8, 9, (257, 300), generator=g).float().to(dev)
    b = torch.randint(-8, 9, (300, 191), generator=g).float().to(dev)
    assert torch.equal(ops.gemm_f32(a, b), (a.double() @ b.double()).float())


@pytest.mark.parametrize("m,k,n", [(300, 257, 129), (1024, 512, 768), (4099, 130, 65), (64, 4096, 64), (1, 7, 1),
                                   (129, 1, 131), (2000, 33, 3), (517, 1000, 300)])
@pytest.mark.parametrize("scale", ["unit", "rows", "tiny", "huge"])
def test_gemm_h3_fused(m, k, n, scale):
    """Fused fp16x3 kernel: fp32-GEMM accuracy against fp64 (same bound family as the split GEMM
    tests), for heterogeneous row / column scales too."""
    from heat_amd import ops

    dev = _dev()
    g = torch.Generator().manual_seed(m + 3 * k + 7 * n)
    a = torch.randn(m, k, generator=g)
    b = torch.randn(k, n, generator=g)
    if scale == "rows":
        a = a * torch.logspace(-6, 6, m).unsqueeze(1)
        b = b * torch.logspace(4, -4, n).unsqueeze(0)
    elif scale == "tiny":
        a, b = a * 1e-20, b * 1e-15
    elif scale == "huge":
        a, b = a * 1e18, b * 1e15
    a, b = a.to(dev), b.to(dev)
    c = ops.gemm_h3(a, b)
    ref = a.double() @ b.double()
    bound = 8 * k * 2.0 ** -24 * (a.abs().double() @ b.abs().double()) + 1e-300
    assert torch.all((c.double() - ref).abs() <= bound), ((c.double() - ref).abs() / bound).max()
    # layouts: a column-major view and a k-contiguous b
    c2 = ops.gemm_h3(a.t().contiguous().t(), b.t().contiguous().t())
    assert torch.equal(c, c2)


# ----------------------------------------------------------------- 256-tile kernels (gemm_tiled.hip)
@pytest.mark.parametrize("m,k,n", [(256, 16, 256), (300, 260, 516), (1000, 33, 4), (4, 4, 4), (513, 1024, 257),
                                   (2048, 20, 300), (8, 4096, 1200)])
@pytest.mark.parametrize("layout", ["nn", "tn", "nt", "tt"])
def test_gemm_f32t_layouts_tails(m, k, n, layout):
    """Exact 256-tile kernel: every layout, K tails (K % 16 != 0 is zeroed in LDS), clamped edge
    rows / columns, against fp64 with the fp32-GEMM bound."""
    from heat_amd import ops

    dev = _dev()
    g = torch.Generator().manual_seed(m + 5 * k + 11 * n)
    a = torch.randn(m, k, generator=g).to(dev)
    b = torch.randn(k, n, generator=g).to(dev)
    A = a if layout[0] == "n" else a.t().contiguous().t()
    B = b if layout[1] == "n" else b.t().contiguous().t()
    c = ops.gemm_f32(A, B)
    ref = a.double() @ b.double()
    assert torch.all((c.double() - ref).abs() <= _bound(a, b)), (c.double() - ref).abs().max()


def test_gemm_f32t_exact_integers_and_alpha_beta():
    from heat_amd import ops

    dev = _dev()
    g = torch.Generator().manual_seed(3)
    a = torch.randint(-8, 9, (600, 272), generator=g).float().to(dev)
    b = torch.randint(-8, 9, (272, 520), generator=g).float().to(dev)
    ref = (a.double() @ b.double()).float()
    assert torch.equal(ops.gemm_f32(a, b), ref)
    c = torch.full((600, 520), 3.0, device=dev)
    ops.gemm_f32(a, b, out=c, accumulate=True, alpha=-1.0)
    assert torch.equal(c, 3.0 - ref)


@pytest.mark.parametrize("m,k,n", [(256, 16, 256), (300, 260, 516), (1000, 33, 5), (1, 7, 1), (513, 1024, 257),
                                   (4099, 130, 65)])
@pytest.mark.parametrize("layout", ["nn", "tn", "nt", "tt"])
def test_gemm_h3t_layouts(m, k, n, layout):
    from heat_amd import ops

    dev = _dev()
    g = torch.Generator().manual_seed(m + 3 * k + 7 * n + len(layout))
    a = (torch.randn(m, k, generator=g) * torch.logspace(-5, 5, m).unsqueeze(1)).to(dev)
    b = (torch.randn(k, n, generator=g) * torch.logspace(3, -3, n).unsqueeze(0)).to(dev)
    A = a if layout[0] == "n" else a.t().contiguous().t()
    B = b if layout[1] == "n" else b.t().contiguous().t()
    c = ops.gemm_h3(A, B)
    ref = a.double() @ b.double()
    bound = 8 * k * 2.0 ** -24 * (a.abs().double() @ b.abs().double()) + 1e-300
    assert torch.all((c.double() - ref).abs() <= bound), ((c.double() - ref).abs() / bound).max()


def test_gemm_h3t_gram_alpha_accumulate_and_nonfinite():
    from heat_amd import ops

    dev = _dev()
    g = torch.Generator().manual_seed(11)
    x = torch.randn(5000, 300, generator=g).to(dev)
    gram = ops.gemm_h3(x.t(), x)
    ref = x.double().t() @ x.double()
    bound = 8 * 5000 * 2.0 ** -24 * (x.abs().double().t() @ x.abs().double())
    assert torch.all((gram.double() - ref).abs() <= bound)
    c = torch.ones(5000, 300, device=dev)
    ops.gemm_h3(x, gram, out=c, alpha=-0.5, accumulate=True)
    r2 = 1 - 0.5 * (x.double() @ gram.double())
    b2 = 8 * 300 * 2.0 ** -24 * 0.5 * (x.abs().double() @ gram.abs().double()) + 1e-6
    assert torch.all((c.double() - r2).abs() <= b2)
    y = x.clone()
    y[3, 4] = float("inf")
    assert ops.gemm_h3(y, gram) is None


@pytest.mark.parametrize("m,k,n", [(2048, 8192, 2048), (300, 5000, 520), (256, 2048, 256), (1000, 65536, 40),
                                   (4, 4096, 4)])
@pytest.mark.parametrize("layout", ["nn", "tn", "nt"])
def test_gemm_f32_split_k(m, k, n, layout, monkeypatch):
    """Few output tiles: K split over slices (one fp32 partial per slice, fixed-order fp64 slice
    sum with alpha / accumulate); same error class as the unsplit GEMM, deterministic, and equal
    to the unsplit kernel within that bound."""
    from heat_amd import ops
    from heat_amd.ops import kernels as K

    dev = _dev()
    g = torch.Generator().manual_seed(m + k + n)
    a = torch.randn(m, k, generator=g).to(dev)
    b = torch.randn(k, n, generator=g).to(dev)
    A = a if layout[0] == "n" else a.t().contiguous().t()
    B = b if layout[1] == "n" else b.t().contiguous().t()
    assert K._splitk_slices(m, n, k, dev) > 1 or m * n > 64 * 65536 or k < 2048
    c = ops.gemm_f32(A, B)
    ref = a.double() @ b.double()
    assert torch.all((c.double() - ref).abs() <= _bound(a, b)), (c.double() - ref).abs().max()
    assert torch.equal(ops.gemm_f32(A, B), c)
    c0 = torch.randn(m, n, generator=g).to(dev)
    c2 = c0.clone()
    ops.gemm_f32(A, B, out=c2, accumulate=True, alpha=-0.5)
    assert torch.all((c2.double() - (c0.double() - 0.5 * ref)).abs() <= 0.5 * _bound(a, b) + 1e-6)
    monkeypatch.setattr(K, "_SPLITK", False)
    cu = ops.gemm_f32(A, B)
    assert torch.all((cu.double() - c.double()).abs() <= 2 * _bound(a, b))


@pytest.mark.parametrize("m,k,n", [(2048, 8192, 2048), (300, 5000, 520)])
def test_gemm_h3_split_k(m, k, n):
    """The fused fp16x3 GEMM with few output tiles takes the split-K path: fp32-GEMM accuracy."""
    from heat_amd import ops
    from heat_amd.ops import kernels as K

    dev = _dev()
    assert K._splitk_slices(m, n, k, dev) > 1
    g = torch.Generator().manual_seed(m + 2 * k + n)
    a = torch.randn(m, k, generator=g).to(dev)
    b = torch.randn(k, n, generator=g).to(dev)
    c = ops.gemm_h3(a, b)
    ref = a.double() @ b.double()
    assert torch.all((c.double() - ref).abs() <= 4 * _bound(a, b)), (c.double() - ref).abs().max()
    c0 = torch.randn(m, n, generator=g).to(dev)
    c2 = c0.clone()
    ops.gemm_h3(a, b, out=c2, alpha=2.0, accumulate=True)
    assert torch.all((c2.double() - (c0.double() + 2 * ref)).abs() <= 8 * _bound(a, b) + 1e-5)


@pytest.mark.parametrize("m,n", [(20000, 1024), (5003, 700), (3000, 513)])
@pytest.mark.parametrize("form", ["tn", "nt"])
@pytest.mark.parametrize("prec", ["highest", "high"])
def test_gram_product_upper_tiles(m, n, form, prec):
    """X^T X and X X^T of one device matrix: upper-triangle tiles + mirror, exactly symmetric, fp32
    GEMM accuracy against fp64."""
    from heat_amd import ops

    dev = _dev()
    g = torch.Generator().manual_seed(m + n)
    x = torch.randn(m, n, generator=g).to(dev)
    if form == "nt":
        x = x.t().contiguous()        # [n, m]: x x^T
    old = torch.get_float32_matmul_precision()
    torch.set_float32_matmul_precision(prec)
    try:
        c = ops.gram_product(x.t(), x) if form == "tn" else ops.gram_product(x, x.t())
    finally:
        torch.set_float32_matmul_precision(old)
    assert c is not None and c.dtype == torch.float32 and c.shape == (n, n)
    xd = x.double()
    ref = xd.t() @ xd if form == "tn" else xd @ xd.t()
    a, b = (x.t(), x) if form == "tn" else (x, x.t())
    assert torch.equal(c, c.t())
    assert torch.all((c.double() - ref).abs() <= _bound(a, b)), (c.double() - ref).abs().max()


def test_matmul_gram_and_cov_route_to_upper_tiles(gpu):
    """ht.matmul(A.T, A) (split 0) and ht.cov reach the Gram path and match fp64."""
    import numpy as np
    import heat_amd as ht
    from heat_amd.core.linalg import basics

    rng = np.random.default_rng(1)
    a = rng.normal(size=(6000, 600)).astype(np.float32)
    A = ht.array(a, split=0, device="gpu")
    calls = []
    orig = basics.fgemm.__globals__.get("_GRAM_MIN_N")
    import heat_amd.ops as _ops
    real = _ops.gram_product

    def spy(x, y):
        r = real(x, y)
        calls.append(r is not None)
        return r

    _ops.gram_product = spy
    try:
        G = ht.matmul(A.T, A).numpy()
        C = ht.cov(ht.array(a.T, split=1, device="gpu")).numpy()
    finally:
        _ops.gram_product = real
    assert orig is not None and any(calls)
    ad = a.astype(np.float64)
    assert np.allclose(G, ad.T @ ad, rtol=1e-4, atol=1e-2)
    assert np.allclose(C, np.cov(ad.T), rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("m,k,n", [(300, 257, 129), (1024, 1024, 1024), (4099, 132, 68), (64, 4096, 64), (1, 7, 1),
                                   (132, 4, 136), (2000, 36, 4), (5000, 256, 700), (128, 20000, 256), (300, 260, 132),
                                   (4100, 128, 100), (1000, 52, 516), (2052, 1028, 260)])
@pytest.mark.parametrize("layout", ["nn", "tn", "nt", "tt"])
@pytest.mark.parametrize("kernel", ["mid128", "mid256", "mid64", "mid128x64", "mid128g2", "s"])
def test_gemm_f32_small_layouts(m, k, n, layout, kernel):
    """128-tile split-K kernels (LDS-DMA gemm_f32m and register-staged gemm_f32s): every operand
    layout, edges, K tails, split-K, alpha / accumulate."""
    from heat_amd import ops

    dev = _dev()
    g = torch.Generator().manual_seed(m * 5 + k * 3 + n)
    a = torch.randn(m, k, generator=g).to(dev)
    b = torch.randn(k, n, generator=g).to(dev)
    A = a if layout[0] == "n" else a.t().contiguous().t()
    B = b if layout[1] == "n" else b.t().contiguous().t()
    c = ops.gemm_f32_small(A, B, kernel=kernel)
    lda = A.stride(0) if A.stride(1) == 1 else A.stride(1)
    ldb = B.stride(0) if B.stride(1) == 1 else B.stride(1)
    if lda % 4 or ldb % 4:
        assert c is None      # 16-byte loads need 4-float leading dimensions: the caller picks another GEMM
        return
    assert c is not None
    ref = a.double() @ b.double()
    assert torch.all((c.double() - ref).abs() <= _bound(a, b)), (c.double() - ref).abs().max()
    base = torch.randn(m, n, generator=g).to(dev)
    out = base.clone()
    ops.gemm_f32_small(A, B, out=out, alpha=-0.5, accumulate=True, kernel=kernel)
    ref2 = base.double() - 0.5 * ref
    assert torch.all((out.double() - ref2).abs() <= _bound(a, b) + 1e-6 * base.abs().double())
    # explicit split-K into a strided column block of a wider C (the Householder update's form)
    wide = torch.randn(m, n + 12, generator=g).to(dev)
    ref3 = wide.double().clone()
    ref3[:, 8: 8 + n] += ref
    ops.gemm_f32_small(A, B, out=wide[:, 8: 8 + n], accumulate=True, slices=3, kernel=kernel)
    err = (wide.double() - ref3).abs()
    assert torch.all(err[:, 8: 8 + n] <= _bound(a, b) + 1e-6 * ref3[:, 8: 8 + n].abs()), kernel
    assert torch.all(err[:, :8] == 0) and torch.all(err[:, 8 + n:] == 0)


@pytest.mark.parametrize("m,k,n", [(6000, 96, 5000), (5996, 64, 4100), (2000, 1000, 1000)])
@pytest.mark.parametrize("layout", ["nn", "tn", "nt", "tt"])
def test_gemm_f32_mid_auto_tile(m, k, n, layout):
    """gemm_f32m with its default tile choice (256 x 128 where the wide tiles fill the GPU): every
    layout, edge tiles in M and N, plain and accumulating."""
    from heat_amd import ops

    dev = _dev()
    g = torch.Generator().manual_seed(m + k + n)
    a = torch.randn(m, k, generator=g).to(dev)
    b = torch.randn(k, n, generator=g).to(dev)
    A = a if layout[0] == "n" else a.t().contiguous().t()
    B = b if layout[1] == "n" else b.t().contiguous().t()
    ref = a.double() @ b.double()
    c = ops.gemm_f32_small(A, B, kernel="mid")
    assert torch.all((c.double() - ref).abs() <= _bound(a, b)), (c.double() - ref).abs().max()
    base = torch.randn(m, n, generator=g).to(dev)
    out = base.clone()
    ops.gemm_f32_small(A, B, out=out, alpha=-1.0, accumulate=True, kernel="mid")
    assert torch.all((out.double() - (base.double() - ref)).abs() <= _bound(a, b) + 1e-6 * base.abs().double())


@pytest.mark.parametrize("m,n,k", [(20000, 3840, 256), (4096, 768, 32), (9000, 300, 256)])
@pytest.mark.parametrize("kernel", ["mid128", "mid256", "mid64", "mid128x64", "mid128g2"])
def test_gemm_f32_mid_update_shape(m, n, k, kernel):
    """The Householder trailing-update form C[:, j:] -= V X on the LDS-DMA 128-tile kernel (C a
    column slice of a row-major matrix, V row-major, X k-major) against fp64."""
    from heat_amd import ops

    dev = _dev()
    g = torch.Generator().manual_seed(m + n + k)
    A = torch.randn(m, n + 256, generator=g).to(dev)
    V = torch.randn(m, k, generator=g).to(dev)
    X = (torch.randn(k, n, generator=g) * 1e-2).to(dev)
    C = A[:, 256:]
    ref = C.double() - V.double() @ X.double()
    left = A[:, :256].clone()
    assert ops.gemm_f32_small(V, X, out=C, alpha=-1.0, accumulate=True, kernel=kernel) is not None
    assert torch.equal(A[:, :256], left)
    assert torch.all((C.double() - ref).abs() <= _bound(V, X) + 1e-6 * ref.abs())


@pytest.mark.parametrize("m,k,n", [(1000, 1000, 1000), (2048, 2048, 2048), (700, 100000, 300), (3000, 3000, 3000),
                                   (129, 70, 4100)])
def test_fgemm_native_plan_products(m, k, n):
    """The products below one wave of 256-tiles run on the kernel / K-slice count of the cost
    model (no library) and keep fp32-GEMM accuracy, with alpha and accumulate."""
    from heat_amd.core.linalg import basics

    dev = _dev()
    g = torch.Generator().manual_seed(m + n + k)
    a = torch.randn(m, k, generator=g).to(dev)
    b = torch.randn(k, n, generator=g).to(dev)
    assert basics._library_better(m, n, k, True)
    kern, sl = basics._native_plan(m, n, k)
    assert kern in ("f32t", "f32s", "f32m64", "f32g2") and sl >= 1
    c = basics.fgemm(a, b)
    ref = a.double() @ b.double()
    assert torch.all((c.double() - ref).abs() <= _bound(a, b)), (kern, sl, (c.double() - ref).abs().max())
    out = torch.ones(m, n, device=dev)
    basics.fgemm(a, b, out=out, alpha=2.0, accumulate=True)
    assert torch.all((out.double() - (1 + 2 * ref)).abs() <= 2 * _bound(a, b) + 1e-6)


@pytest.mark.parametrize("m,n", [(1000, 260), (4099, 1000), (2048, 1536), (300, 4), (777, 513)])
@pytest.mark.parametrize("layout", ["nn", "tn", "nt", "tt"])
@pytest.mark.parametrize("kernel", ["f32", "f32_split", "h3"])
def test_gemm_b_upper_triangular(m, n, layout, kernel):
    """``b_upper``: B square upper triangular, output column tile n0 contracts only k < n0 + 256.
    fp64-bounded like the full product, every operand layout, N not a multiple of 256, split-K
    slices wholly beyond a tile's clipped K (their partials must be zero), and the result equal
    to the full kernel's where every skipped product is a multiplication by zero."""
    from heat_amd import ops

    dev = _dev()
    g = torch.Generator().manual_seed(m + 31 * n)
    a = torch.randn(m, n, generator=g).to(dev)
    b = torch.triu(torch.randn(n, n, generator=g) + 2 * torch.eye(n)).to(dev)
    A = a if layout[0] == "n" else a.t().contiguous().t()
    B = b if layout[1] == "n" else b.t().contiguous().t()
    ref = a.double() @ b.double()
    if kernel == "h3":
        c = ops.gemm_h3(A, B, b_upper=True)
        full = ops.gemm_h3(A, B)
        bound = 8 * n * 2.0 ** -24 * (a.abs().double() @ b.abs().double()) + 1e-30
    else:
        sl = 4 if kernel == "f32_split" else None
        c = ops.gemm_f32(A, B, b_upper=True, slices=sl)
        full = ops.gemm_f32(A, B, slices=sl)
        bound = _bound(a, b)
    err = (c.double() - ref).abs()
    assert torch.all(err <= bound), err.max()
    if kernel != "h3":
        # skipping exact zeros changes no partial sum of a k-ordered chain: bit-identical
        assert torch.equal(c, full)
    # alpha / accumulate ride along
    out = torch.ones(m, n, device=dev)
    ops.gemm_f32(A, B, out=out, accumulate=True, alpha=0.5, b_upper=True)
    assert torch.allclose(out.double(), 1 + 0.5 * ref, rtol=1e-5, atol=1e-3 * n ** 0.5)
