"""Numerics of the native CDNA4 kernels against plain PyTorch fp32/fp64 references (GPU only)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from heat_amd import ops

    assert ops.available(), "native library must load on a GPU box"
    return torch.device("cuda", 0)


@pytest.mark.parametrize("n,k,f", [(1000, 7, 3), (4096, 128, 16), (5000, 300, 32), (20000, 1024, 64),
                                   (3333, 100, 100), (777, 65, 128)])
def test_kmeans_assign(n, k, f):
    from heat_amd import ops

    dev = _dev()
    g = torch.Generator(device="cpu").manual_seed(n + k + f)
    X = torch.randn(n, f, generator=g).to(dev)
    C = torch.randn(k, f, generator=g).to(dev)
    lab, mind = ops.kmeans_assign(X, C)
    Xd, Cd = X.double(), C.double()
    d = torch.cdist(Xd, Cd) ** 2
    ref_min, ref_lab = d.min(1)
    # labels may only differ on numerical near-ties
    chosen = d.gather(1, lab.long().unsqueeze(1)).squeeze(1)
    assert torch.all(chosen - ref_min <= 1e-4 * (1 + ref_min)), "assigned centroid not (near-)minimal"
    assert (lab.long() == ref_lab).float().mean() > 0.999
    assert torch.allclose(mind.double(), ref_min, rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("n,k,f", [(1000, 7, 3), (4096, 128, 16), (5000, 300, 32), (20000, 1024, 64),
                                   (3333, 100, 100), (777, 65, 128), (70000, 1000, 64)])
@pytest.mark.parametrize("scale", [1.0, 1e-3, 1e4])
def test_kmeans_assign_f16x3(n, k, f, scale):
    """fp16x3 split assignment: the chosen centroid is minimal up to fp32-GEMM rounding."""
    from heat_amd import ops

    dev = _dev()
    g = torch.Generator(device="cpu").manual_seed(n + 3 * k + f)
    X = (torch.randn(n, f, generator=g) * scale).to(dev)
    C = (torch.randn(k, f, generator=g) * scale).to(dev)
    packed = ops.kmeans_pack_points(X)
    assert packed is not None
    lab, mind = ops.kmeans_assign(X, C, packed=packed)
    Xd, Cd = X.double(), C.double()
    d = torch.cdist(Xd, Cd) ** 2
    ref_min, ref_lab = d.min(1)
    chosen = d.gather(1, lab.long().unsqueeze(1)).squeeze(1)
    tol = 2e-6 * ((Xd * Xd).sum(1) + (Cd * Cd).sum(1).max())
    assert torch.all(chosen - ref_min <= tol), (chosen - ref_min - tol).max()
    assert (lab.long() == ref_lab).float().mean() > 0.995
    assert torch.allclose(mind.double(), ref_min, rtol=1e-4, atol=1e-4 * scale * scale * f)


def _hetero(n, k, f, seed, span=(-4.0, 4.0)):
    """Centroid norms log-uniform over 10^span (1e-4 .. 1e4) within ONE call; every point sits
    near a random centroid (noise 20% of that centroid's norm), so points near the tiny centroids
    need the tiny centroids' products at full relative precision."""
    g = torch.Generator(device="cpu").manual_seed(seed)
    lo, hi = span
    norms = 10.0 ** (lo + (hi - lo) * torch.rand(k, generator=g, dtype=torch.float64))
    C = torch.randn(k, f, generator=g, dtype=torch.float64)
    C = C / C.norm(dim=1, keepdim=True) * norms[:, None]
    owner = torch.randint(0, k, (n,), generator=g)
    X = C[owner] + 0.2 * norms[owner, None] * torch.randn(n, f, generator=g, dtype=torch.float64) / f ** 0.5
    return X.float(), C.float()


def _local_minimality(X, C, lab):
    """chosen - best <= tol_i with tol_i LOCAL to point i: it scales with |x_i|^2 and the norms of
    the two contenders only (not with the largest centroid), i.e. fp32-GEMM relative accuracy per
    centroid."""
    Xd, Cd = X.double(), C.double()
    d = torch.cdist(Xd, Cd) ** 2
    ref_min, ref_lab = d.min(1)
    chosen = d.gather(1, lab.long().unsqueeze(1)).squeeze(1)
    cn = (Cd * Cd).sum(1)
    tol = 4e-6 * ((Xd * Xd).sum(1) + cn[lab.long()] + cn[ref_lab])
    bad = chosen - ref_min > tol
    return bad, d, ref_min, ref_lab


@pytest.mark.parametrize("mode", ["resident_all", "chunked", "certified"])
@pytest.mark.parametrize("n,k,f", [(20000, 1024, 64), (5000, 300, 32), (3333, 200, 100), (9000, 500, 16)])
def test_kmeans_assign_f16x3_heterogeneous_centroids(n, k, f, mode, monkeypatch):
    """Centroid norms spanning 1e-4..1e4 in one call: per-centroid scales keep every centroid at
    fp32-GEMM relative accuracy (a shared scale lost up to 27 bits on the smallest ones)."""
    from heat_amd import ops

    dev = _dev()
    monkeypatch.setattr(ops.kernels, "_H3_RESIDENT", mode == "resident_all")
    monkeypatch.setattr(ops.kernels, "_H3_RESIDENT_ALL", mode == "resident_all")
    X, C = _hetero(n, k, f, seed=n + k + f)
    X, C = X.to(dev), C.to(dev)
    packed = ops.kmeans_pack_points(X)
    lab, mind = ops.kmeans_assign(X, C, want_mind=mode != "certified", packed=packed,
                                  certified=mode == "certified")
    bad, d, ref_min, ref_lab = _local_minimality(X, C, lab)
    assert not bad.any(), int(bad.sum())
    assert (lab.long() == ref_lab).float().mean() > 0.999
    if mind is not None:
        assert torch.all((mind.double() - ref_min).abs() <= 1e-4 * ref_min + 4e-6 * (X.double() ** 2).sum(1))


def test_knn_topk_heterogeneous(gpu):
    from heat_amd import ops

    X, C = _hetero(3000, 4000, 32, seed=5)
    X, C = X.cuda(), C.cuda()
    dist, idx = ops.knn_topk(X, C, 4)
    d = torch.cdist(X.double(), C.double()) ** 2
    ref, _ = d.topk(4, dim=1, largest=False)
    got = d.gather(1, idx.long())
    tol = 4e-6 * ((X.double() ** 2).sum(1, keepdim=True) + (C.double() ** 2).sum(1)[idx.long()])
    assert torch.all(got - ref <= tol)


@pytest.mark.parametrize("mode", ["resident_all", "chunked"])
@pytest.mark.parametrize("n,k,f", [(5000, 300, 32), (70000, 1500, 64), (3333, 700, 100), (9000, 2100, 16)])
def test_kmeans_assign_f16x3_kernels(n, k, f, mode, monkeypatch):
    """Both fp16x3 assignment kernels: LDS-resident centroids (in phases past the LDS capacity,
    carrying the running best through global memory) and chunk-staged; same labels and distances."""
    from heat_amd import ops

    dev = _dev()
    monkeypatch.setattr(ops.kernels, "_H3_RESIDENT", mode == "resident_all")
    monkeypatch.setattr(ops.kernels, "_H3_RESIDENT_ALL", mode == "resident_all")
    g = torch.Generator(device="cpu").manual_seed(n + k + f)
    X = torch.randn(n, f, generator=g).to(dev)
    C = torch.randn(k, f, generator=g).to(dev)
    C[k - 1] = C[3]          # exact duplicate: the lower index must win
    packed = ops.kmeans_pack_points(X)
    lab, mind = ops.kmeans_assign(X, C, packed=packed)
    d = torch.cdist(X.double(), C.double()) ** 2
    ref_min, ref_lab = d.min(1)
    chosen = d.gather(1, lab.long().unsqueeze(1)).squeeze(1)
    tol = 2e-6 * ((X.double() ** 2).sum(1) + (C.double() ** 2).sum(1).max())
    assert torch.all(chosen - ref_min <= tol)
    assert (lab.long() == ref_lab).float().mean() > 0.995
    assert not torch.any(lab == k - 1)
    assert torch.allclose(mind.double(), ref_min, rtol=1e-4, atol=1e-4 * f)


@pytest.mark.parametrize("n,k,f", [(1000, 7, 3), (5000, 300, 32), (70000, 1024, 64), (3333, 100, 100),
                                   (777, 65, 128), (40000, 16, 18)])
@pytest.mark.parametrize("data", ["normal", "near_centroids", "ties"])
def test_kmeans_assign_certified(n, k, f, data):
    """One-term filter + 3-term re-check: same minimality guarantee as the full fp16x3 kernel."""
    from heat_amd import ops

    dev = _dev()
    g = torch.Generator(device="cpu").manual_seed(n + 7 * k + f)
    C = torch.randn(k, f, generator=g)
    if data == "normal":
        X = torch.randn(n, f, generator=g)
    elif data == "near_centroids":   # tight clusters: mostly clear wins, a few far points
        X = C[torch.randint(0, k, (n,), generator=g)] + 0.05 * torch.randn(n, f, generator=g)
    else:                            # exact duplicates of centroids -> exact ties everywhere
        C[1::2] = C[0::2][: C[1::2].shape[0]]
        X = C[torch.randint(0, k, (n,), generator=g)].clone()
    X, C = X.to(dev), C.to(dev)
    packed = ops.kmeans_pack_points(X)
    lab, mind = ops.kmeans_assign(X, C, want_mind=False, packed=packed, certified=True)
    assert mind is None
    nre = int(ops.kmeans_assign.last_rechecked.item())
    assert 0 <= nre <= n
    Xd, Cd = X.double(), C.double()
    d = torch.cdist(Xd, Cd) ** 2
    ref_min, _ = d.min(1)
    chosen = d.gather(1, lab.long().unsqueeze(1)).squeeze(1)
    tol = 2e-6 * ((Xd * Xd).sum(1) + (Cd * Cd).sum(1).max())
    assert torch.all(chosen - ref_min <= tol), (chosen - ref_min - tol).max()
    full, _ = ops.kmeans_assign(X, C, want_mind=True, packed=packed)
    assert (lab == full).float().mean() > 0.999
    if data == "near_centroids":
        assert nre < n // 10, nre


def test_kmeans_fast_matches_exact_fit(gpu):
    import heat_amd as ht

    ht.random.seed(3)
    x = ht.random.randn(60000, 32, split=0)
    res = []
    for prec in ("exact", "fast"):
        km = ht.cluster.KMeans(n_clusters=64, init="random", max_iter=5, tol=None, random_state=9)
        km.precision = prec
        km.fit(x)
        res.append(km.cluster_centers_.larray)
    assert torch.allclose(res[0], res[1], atol=1e-3)


@pytest.mark.parametrize("n,k,f", [(1000, 7, 3), (50000, 1024, 64), (12345, 33, 100), (4096, 8, 18)])
def test_kmeans_update(n, k, f):
    from heat_amd import ops

    dev = _dev()
    g = torch.Generator(device="cpu").manual_seed(n)
    X = torch.randn(n, f, generator=g).to(dev)
    lab = torch.randint(0, k, (n,), generator=g).to(dev).to(torch.int32)
    sums, counts = ops.kmeans_update(X, lab, k)
    ref = torch.zeros(k, f, dtype=torch.float64, device=dev).index_add_(0, lab.long(), X.double())
    rc = torch.bincount(lab.long(), minlength=k).double()
    assert torch.allclose(sums.double(), ref, rtol=1e-4, atol=1e-3)
    assert torch.equal(counts.double(), rc)


@pytest.mark.parametrize("n,k,f,skew", [(1_000_000, 1024, 64, False), (300_000, 64, 64, True), (70_001, 5, 17, True),
                                         (200_000, 3000, 8, False), (12345, 33, 100, False)])
def test_kmeans_update_deterministic(n, k, f, skew):
    """The default update is order-independent: repeated calls (different scheduling each time) give
    bit-identical sums, which match an fp64 reference to fp32 rounding. Skewed labels (a few huge
    clusters spanning many gather ranges, empty clusters) exercise the segment walk."""
    from heat_amd import ops

    dev = _dev()
    g = torch.Generator(device="cpu").manual_seed(n + k)
    X = torch.randn(n, f, generator=g).to(dev)
    if skew:
        lab = (torch.randn(n, generator=g).abs() * k / 6).long().clamp(max=k - 1)
        lab[lab == 1] = 0          # an empty cluster
    else:
        lab = torch.randint(0, k, (n,), generator=g)
    lab = lab.to(dev).to(torch.int32)
    sums, counts = ops.kmeans_update(X, lab, k)
    for _ in range(3):
        s2, c2 = ops.kmeans_update(X, lab, k)
        assert torch.equal(s2, sums) and torch.equal(c2, counts)
    ref = torch.zeros(k, f, dtype=torch.float64, device=dev).index_add_(0, lab.long(), X.double())
    rc = torch.bincount(lab.long(), minlength=k).double()
    assert torch.equal(counts.double(), rc)
    bound = 1e-6 * torch.zeros(k, f, dtype=torch.float64, device=dev).index_add_(0, lab.long(), X.double().abs()) \
        + 1e-6
    assert torch.all((sums.double() - ref).abs() <= 4 * bound), ((sums.double() - ref).abs() / bound).max()


def test_kmeans_fit_bit_reproducible():
    """Two fits with the same seed give bit-identical centroids and labels (deterministic update)."""
    import heat_amd as ht

    _dev()
    ht.use_device("gpu")
    ht.random.seed(5)
    x = ht.random.randn(400_000, 32, split=0)
    out = []
    for _ in range(2):
        km = ht.cluster.KMeans(n_clusters=256, init="random", max_iter=8, tol=None, random_state=11)
        km.fit(x)
        out.append((km.cluster_centers_.larray.clone(), km.labels_.larray.clone()))
    assert torch.equal(out[0][0], out[1][0])
    assert torch.equal(out[0][1], out[1][1])


@pytest.mark.parametrize("k,f,packed", [(3, 5, True), (3, 5, False), (1024, 64, True), (1024, 64, False),
                                         (5000, 100, False), (7, 1, True)])
def test_kmeans_finalize(k, f, packed):
    """Native Lloyd epilogue vs fp64 torch: means, empty clusters keep their centroid, squared shift
    (the last-block reduction resets its arrival counter: three launches in a row agree)."""
    from heat_amd import ops

    dev = _dev()
    g = torch.Generator(device="cpu").manual_seed(k * f)
    C = torch.randn(k, f, generator=g).to(dev)
    sums = (torch.randn(k, f, generator=g) * 50).to(dev)
    counts = torch.randint(0, 40, (k,), generator=g).float().to(dev)
    counts[0] = 0.0
    ref = torch.where(counts.double().unsqueeze(1) > 0, sums.double() / counts.double().clamp(min=1).unsqueeze(1),
                      C.double())
    ref_shift = float(((C.double() - ref.float().double()) ** 2).sum())
    for _ in range(3):
        if packed:
            pk = torch.cat([sums.reshape(-1).double(), counts.double()])
            newC, shift = ops.kmeans_finalize(pk, C)
        else:
            newC, shift = ops.kmeans_finalize(None, C, sums=sums, counts=counts)
        assert torch.allclose(newC.double(), ref, rtol=1e-6, atol=1e-6)
        assert torch.equal(newC[0], C[0])
        assert abs(float(shift) - ref_shift) <= 1e-9 * max(1.0, ref_shift)


@pytest.mark.parametrize("shape,axis", [((10_000_003,), None), ((1000, 999), None), ((1000, 999), 0),
                                        ((1000, 999), 1), ((3, 1000, 4), 1), ((513, 1024), 0), ((7, 5), 1)])
def test_moments(shape, axis):
    from heat_amd import ops

    dev = _dev()
    g = torch.Generator(device="cpu").manual_seed(len(shape))
    x = (torch.randn(*shape, generator=g) * 3 + 100).to(dev)
    n, mu, m2 = ops.moments(x, axis)
    xd = x.double()
    if axis is None:
        rv, rm = torch.var_mean(xd, correction=0)
    else:
        rv, rm = torch.var_mean(xd, dim=axis, correction=0)
    assert torch.allclose(mu, rm, rtol=1e-6, atol=1e-5)
    assert torch.allclose(m2 / n, rv, rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("shape,axis", [((3_000_000,), None), ((1000, 5000), None), ((300, 70001), 1),
                                        ((70001, 300), 0), ((200_000, 3), 0), ((5, 1_000_001), 1),
                                        ((64, 50, 33), 1), ((1000, 1001), 0), ((1000, 1001), 1),
                                        ((50_000, 1000), 1), ((100_000, 4), 1), ((33, 1024), 1), ((7, 8), 1)])
@pytest.mark.parametrize("final", ["mean", "var", "std"])
def test_moments_fused_final(shape, axis, final):
    """ONE launch per call: the per-chunk partials are merged by each output's last-arriving block
    (fixed chunk order, so repeated calls are bit-identical) and the fp32 result written directly."""
    from heat_amd import ops

    dev = _dev()
    g = torch.Generator(device="cpu").manual_seed(sum(shape) + (axis or 0))
    x = (torch.randn(*shape, generator=g) * 3 + 100).to(dev)
    ddof = 1 if final != "mean" else 0
    r = ops.moments(x, axis, final, ddof)
    assert r.dtype == torch.float32
    xd = x.double()
    if axis is None:
        rv, rm = torch.var_mean(xd, correction=ddof)
    else:
        rv, rm = torch.var_mean(xd, dim=axis, correction=ddof)
    ref = {"mean": rm, "var": rv, "std": rv.sqrt()}[final]
    assert r.shape == ref.shape
    assert torch.allclose(r.double(), ref, rtol=2e-6, atol=1e-6), (r.double() - ref).abs().max()
    for _ in range(3):
        assert torch.equal(ops.moments(x, axis, final, ddof), r)
    # the triples path agrees with the fused one
    n, mu, m2 = ops.moments(x, axis)
    if final == "mean":
        assert torch.equal(mu.float(), r)


def test_moments_concurrent_streams():
    """Fused moments on two streams at once: each (device, stream) has its own arrival counters,
    so the two kernels' ticket trees never share a word."""
    from heat_amd import ops

    dev = _dev()
    g = torch.Generator(device="cpu").manual_seed(3)
    xs = [(torch.randn(3_000_000, generator=g) * (i + 1) + 10 * i).to(dev) for i in range(2)]
    ys = [(torch.randn(20_000, 300, generator=g) + i).to(dev) for i in range(2)]
    streams = [torch.cuda.Stream(device=dev) for _ in range(2)]
    torch.cuda.synchronize()
    res = [None, None]
    for _ in range(5):
        for i, st in enumerate(streams):
            with torch.cuda.stream(st):
                res[i] = (ops.moments(xs[i], None, "var"), ops.moments(ys[i], 0, "mean"))
        torch.cuda.synchronize()
        for i in range(2):
            assert abs(res[i][0].item() - xs[i].double().var(correction=0).item()) < 1e-5 * (1 + (i + 1) ** 2)
            assert torch.allclose(res[i][1].double(), ys[i].double().mean(0), rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("rows,length,ld", [(5000, 1021, 1024), (777, 7, 8), (64, 1024, 1024), (3, 5, 12)])
@pytest.mark.parametrize("kind", [1, 2, 3])
def test_moments_short_rows_padded_stride(rows, length, ld, kind):
    """The short-row pipeline (a few workgroups per CU, next row in flight, register mean shift)
    on rows of `length` inside a padded row stride `ld` (16-byte aligned rows, scalar tail of
    length % 4 elements) through the C ABI directly: mean / var / std against fp64."""
    import ctypes

    from heat_amd import ops
    from heat_amd.ops import kernels as K

    dev = _dev()
    g = torch.Generator(device="cpu").manual_seed(rows + length)
    buf = (torch.randn(rows, ld, generator=g) * 2 + 50).to(dev)
    x = buf[:, :length]
    out = torch.empty(rows, dtype=torch.float32, device=dev)
    part = torch.empty(rows * 3, dtype=torch.float64, device=dev)
    L = ops.lib()
    st = ctypes.c_void_p(ops.stream_ptr(dev))
    ops.check(L.ha_moments_rows(K._ptr(buf), rows, length, ld, 1, K._ptr(part), K._ptr(out), kind, 0.0, None, st),
              "ha_moments_rows")
    xd = x.double()
    ref = {1: xd.mean(1), 2: xd.var(1, correction=0), 3: xd.var(1, correction=0).sqrt()}[kind]
    assert torch.allclose(out.double(), ref, rtol=2e-6, atol=1e-6), (out.double() - ref).abs().max()
    # triples (kind 0) of the same rows
    trip = torch.empty(rows, 3, dtype=torch.float64, device=dev)
    ops.check(L.ha_moments_rows(K._ptr(buf), rows, length, ld, 1, K._ptr(part), K._ptr(trip), 0, 0.0, None, st),
              "ha_moments_rows")
    assert torch.all(trip[:, 0] == length)
    assert torch.allclose(trip[:, 1], xd.mean(1), rtol=1e-9, atol=1e-9)
    assert torch.allclose(trip[:, 2] / length, xd.var(1, correction=0), rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("shape,axis", [((4_000_000, 64), 0), ((64, 4_000_000), None), ((2000, 3000), 0)])
def test_moments_handoff_fresh_each_call(shape, axis):
    """The fused epilogue hands partials between blocks with write-through stores and a ticket
    (no per-block release fence). Refill the SAME input buffer with new values before every call
    (the workspaces come back from the caching allocator at the same addresses), so a stale
    partial from the previous call would show up as a wrong result."""
    from heat_amd import ops

    dev = _dev()
    x = torch.empty(*shape, device=dev)
    g = torch.Generator(device=dev).manual_seed(5)
    for it in range(12):
        x.normal_(mean=float(it * 7 - 30), std=1.0 + it, generator=g)
        r = ops.moments(x, axis, "var", 0)
        xd = x.double()
        rv = torch.var(xd, correction=0) if axis is None else torch.var(xd, dim=axis, correction=0)
        assert torch.allclose(r.double(), rv, rtol=1e-5, atol=1e-6), (it, (r.double() - rv).abs().max())
        m = ops.moments(x, axis, "mean")
        rm = xd.mean() if axis is None else xd.mean(axis)
        assert torch.allclose(m.double(), rm, rtol=1e-6, atol=1e-5), (it, (m.double() - rm).abs().max())


@pytest.mark.parametrize("exact", [False, True])
@pytest.mark.parametrize("metric", ["euclidean", "sqeuclidean", "gaussian", "manhattan"])
@pytest.mark.parametrize("m,n,f", [(100, 50, 3), (1000, 777, 18), (257, 300, 128), (64, 64, 200)])
def test_cdist(metric, m, n, f, exact):
    from heat_amd import ops

    dev = _dev()
    g = torch.Generator(device="cpu").manual_seed(m * n)
    X = torch.rand(m, f, generator=g).to(dev)
    Y = torch.rand(n, f, generator=g).to(dev)
    out = ops.cdist(X, Y, metric, sigma=2.0, exact=exact)
    Xd, Yd = X.double(), Y.double()
    if metric == "manhattan":
        ref = torch.cdist(Xd, Yd, p=1)
    else:
        d2 = torch.cdist(Xd, Yd) ** 2
        ref = {"euclidean": d2.sqrt(), "sqeuclidean": d2, "gaussian": torch.exp(-d2 / 8.0)}[metric]
    tol = 2e-3 if (metric == "euclidean" and not exact) else 1e-4
    assert torch.allclose(out.double(), ref, rtol=tol, atol=tol)
    if exact and metric == "euclidean":
        # identical rows: exactly zero distance (no cancellation)
        self_d = ops.cdist(X, X, metric, exact=True)
        assert torch.all(torch.diagonal(self_d) == 0)


@pytest.mark.parametrize("metric", ["euclidean", "manhattan"])
@pytest.mark.parametrize("m,n,f", [(300, 129, 37), (129, 1000, 18), (1, 5, 3), (200, 257, 65)])
def test_cdist_exact_strided_views(metric, m, n, f):
    """Exact (difference) kernel on row-strided views whose LAST row ends at the allocation's end
    (the tile's buffer range must stop at column f of the last row), into an output with a row
    stride that is not a multiple of 4 (scalar store path)."""
    from heat_amd import ops

    dev = _dev()
    g = torch.Generator(device="cpu").manual_seed(m + n + f)
    bx = torch.rand(m * (f + 5), generator=g)[: (m - 1) * (f + 5) + f].to(dev)
    by = torch.rand(n * (f + 3), generator=g)[: (n - 1) * (f + 3) + f].to(dev)
    X = torch.as_strided(bx, (m, f), (f + 5, 1))
    Y = torch.as_strided(by, (n, f), (f + 3, 1))
    big = torch.full((m, n + 3), -1.0, device=dev)
    out = big[:, :n]
    ops.cdist(X, Y, metric, exact=True, out=out)
    Xd, Yd = X.double(), Y.double()
    ref = torch.cdist(Xd, Yd, p=1) if metric == "manhattan" else torch.cdist(Xd, Yd)
    assert torch.allclose(out.double(), ref, rtol=1e-5, atol=1e-5)
    assert torch.all(big[:, n:] == -1.0)


@pytest.mark.parametrize("precision", ["f16x3", "fp32"])
@pytest.mark.parametrize("metric", ["euclidean", "sqeuclidean", "gaussian"])
@pytest.mark.parametrize("m,n,f", [(100, 50, 3), (1000, 777, 18), (513, 640, 64), (130, 1100, 96), (257, 300, 128),
                                   (300, 129, 200), (40, 2000, 1000)])
@pytest.mark.parametrize("scale", [1.0, 1e-3, 1e3])
def test_cdist_expansion(metric, m, n, f, precision, scale):
    """Quadratic-expansion kernels: squared distances within fp32-GEMM rounding of the exact ones."""
    from heat_amd import ops

    dev = _dev()
    g = torch.Generator(device="cpu").manual_seed(m + n + f)
    X = (torch.randn(m, f, generator=g) * scale).to(dev)
    Y = (torch.randn(n, f, generator=g) * scale + 0.5 * scale).to(dev)
    sigma = 2.0 * scale * (f ** 0.5)
    out = ops.cdist(X, Y, metric, sigma=sigma, precision=precision).double()
    Xd, Yd = X.double(), Y.double()
    d2 = torch.cdist(Xd, Yd) ** 2
    bound = 1e-5 * ((Xd * Xd).sum(1, keepdim=True) + (Yd * Yd).sum(1))   # cancellation scale
    if metric == "sqeuclidean":
        assert torch.all((out - d2).abs() <= bound + 1e-30)
    elif metric == "euclidean":
        assert torch.all((out ** 2 - d2).abs() <= 2 * bound + 1e-30)
    else:
        ref = torch.exp(-d2 / (2 * sigma * sigma))
        assert torch.allclose(out, ref, rtol=1e-4, atol=1e-5)


def test_cdist_stream_matches_full(gpu):
    import heat_amd as ht

    ht.random.seed(11)
    x = ht.random.rand(3000, 40, split=0)
    full = ht.spatial.cdist(x, x, quadratic_expansion=True).larray
    got = torch.empty_like(full)

    def consume(d, i, j):
        got[i: i + d.shape[0], j: j + d.shape[1]] = d

    for tile in (1024, 1000):  # 1000 is rounded down to a multiple of 128 rows
        got.zero_()
        ht.spatial.cdist_stream(x, x, consume, tile=tile)
        assert torch.allclose(got, full, atol=1e-5)


def test_cdist_packed_row_slices(gpu):
    """Packed operands sliced at multiples of 128 rows == packing the slice itself."""
    from heat_amd import ops

    dev = _dev()
    g = torch.Generator(device="cpu").manual_seed(3)
    X = torch.randn(1000, 128, generator=g).to(dev)
    Y = torch.randn(700, 128, generator=g).to(dev)
    px, py = ops.cdist_pack(X), ops.cdist_pack(Y)
    assert px.planes.shape[0] == 1024 and px.n == 1000
    full = ops.cdist(X, Y, packed_x=px, packed_y=py)
    part = ops.cdist(X[256:900], Y[384:], packed_x=px.rows(256, 900), packed_y=py.rows(384, 700))
    assert torch.allclose(part, full[256:900, 384:], atol=1e-6)
    with pytest.raises(ValueError):
        px.rows(100, 200)


def test_threefry_bit_exact():
    """Device Threefry kernel == host torch implementation, bit for bit (uniform / int)."""
    import heat_amd as ht

    _dev()
    for dtype in (ht.float32, ht.float64):
        for state in (0, 0xFFFFFFFFFFFFFFF0, (1 << 128) - 16):
            ht.random.set_state(("Threefry", 12345, state))
            a = ht.random.rand(1001, 3, dtype=dtype, device="cpu")
            ht.random.set_state(("Threefry", 12345, state))
            b = ht.random.rand(1001, 3, dtype=dtype, device="gpu")
            assert torch.equal(a.larray, b.larray.cpu())
    for dtype in (ht.int32, ht.int64):
        ht.random.set_state(("Threefry", 99, 5))
        a = ht.random.randint(-7, 1000, size=(333, 7), dtype=dtype, device="cpu")
        ht.random.set_state(("Threefry", 99, 5))
        b = ht.random.randint(-7, 1000, size=(333, 7), dtype=dtype, device="gpu")
        assert torch.equal(a.larray, b.larray.cpu())
    ht.random.set_state(("Threefry", 3, 0))
    a = ht.random.randn(2000, device="cpu")
    ht.random.set_state(("Threefry", 3, 0))
    b = ht.random.randn(2000, device="gpu")
    # the Kundu transform goes through device transcendentals: equal to a few ulp
    assert torch.allclose(a.larray, b.larray.cpu(), rtol=1e-4, atol=1e-4)


def test_randn_fast_transform_parity_and_distribution():
    """The hardware-log/exp Kundu transform (+ precise table near u = 1) stays within the host
    parity bound on EVERY one of 1e7 samples, and the sample moments / KS statistic match the
    host path."""
    import heat_amd as ht

    _dev()
    n = 10_000_000
    ht.random.set_state(("Threefry", 2024, 77))
    a = ht.random.randn(n, device="cpu").larray.double()
    ht.random.set_state(("Threefry", 2024, 77))
    b = ht.random.randn(n, device="gpu").larray.cpu().double()
    err = ((a - b).abs() / (1 + a.abs())).max().item()
    assert err < 1e-4, err
    assert abs(b.mean().item() - a.mean().item()) < 1e-6
    assert abs(b.var().item() / a.var().item() - 1) < 1e-5
    # two-sample KS statistic between host and device samples (identical up to rounding)
    sa, sb = torch.sort(a).values, torch.sort(b).values
    grid = torch.linspace(-5, 5, 2001, dtype=torch.float64)
    ks = (torch.searchsorted(sa, grid).double() - torch.searchsorted(sb, grid).double()).abs().max().item() / n
    assert ks < 1e-5, ks


def test_kmeans_fit_gpu(gpu):
    import heat_amd as ht

    ht.random.seed(1)
    # well separated blobs
    centers = torch.tensor([[0.0, 0.0], [10.0, 10.0], [-10.0, 10.0], [10.0, -10.0]])
    pts = torch.cat([c + torch.randn(500, 2) for c in centers])
    x = ht.array(pts, split=0, device="gpu")
    km = ht.cluster.KMeans(n_clusters=4, init="kmeans++", max_iter=50, random_state=2)
    km.fit(x)
    got = km.cluster_centers_.larray.cpu()
    d = torch.cdist(got, centers)
    assert torch.all(d.min(1).values < 0.5)
    assert km.labels_.shape == (2000, 1)


@pytest.mark.parametrize("m,n", [(1000, 3), (70001, 16), (513, 130), (300001, 20), (4097, 64), (100, 33)])
def test_lasso_prepare(m, n):
    from heat_amd import ops

    dev = _dev()
    X = torch.randn(m, n, generator=torch.Generator().manual_seed(m)).to(dev)
    XT, colsq = ops.lasso_prepare(X)
    assert torch.equal(XT, X.t().contiguous())
    assert torch.allclose(colsq.double(), (X.double() ** 2).sum(0), rtol=1e-5)


@pytest.mark.parametrize("m,n", [(1, 1), (1000, 3), (70001, 16), (300001, 23), (4097, 7), (100, 40)])
def test_lasso_gram_matches_fp64(gpu, m, n):
    from heat_amd import ops

    g = torch.Generator().manual_seed(m + n)
    X = torch.randn(m, n, generator=g)
    y = torch.randn(m, generator=g)
    G = ops.lasso_gram(X.cuda(), y.cuda()).cpu()
    A = torch.cat([X, y[:, None]], 1).double()
    ref = A.T @ A
    assert torch.allclose(G, ref, rtol=1e-5, atol=1e-6 * m), (G - ref).abs().max()


@pytest.mark.parametrize("n", [5, 64, 65, 130, 700, 1500])
@pytest.mark.parametrize("tol", [None, 1e-6])
def test_lasso_cd_device_matches_host(gpu, n, tol):
    from heat_amd import ops

    g = torch.Generator().manual_seed(n)
    X = torch.randn(4 * n + 50, n, generator=g, dtype=torch.float64)
    X /= X.pow(2).mean(0).sqrt()
    y = X @ torch.randn(n, generator=g, dtype=torch.float64)
    G = torch.cat([X, y[:, None]], 1)
    G = G.T @ G / X.shape[0]
    res = []
    for dev in ("cpu", "cuda"):
        Gd = G.to(dev)
        th = torch.zeros(n, dtype=torch.float64, device=dev)
        it = ops.lasso_cd(Gd[:n, :n], Gd[:n, n].contiguous(), 0.02, 25, tol, th)
        res.append((it, th.cpu()))
    assert res[0][0] == res[1][0]
    assert torch.allclose(res[0][1], res[1][1], atol=1e-9)


@pytest.mark.parametrize("n", [16, 200])
def test_lasso_gram_solver_matches_sweep(gpu, monkeypatch, n):
    import heat_amd as ht

    ht.random.seed(5)
    x = ht.random.randn(50000, n)
    x = x / ht.sqrt(ht.mean(x ** 2, axis=0))
    y = ht.matmul(x, ht.random.randn(n, 1)) + 0.05 * ht.random.randn(50000, 1)
    res = []
    for solver in ("sweep", "gram"):
        monkeypatch.setenv("HEAT_LASSO_SOLVER", solver)
        est = ht.regression.Lasso(lam=0.01, max_iter=30, tol=None)
        est.fit(x, y)
        res.append(est.theta.larray.cpu().double())
    assert torch.allclose(res[0], res[1], atol=2e-4), (res[0] - res[1]).abs().max()


def test_lasso_graph_replay_matches_eager(gpu, monkeypatch):
    import heat_amd as ht

    ht.random.seed(4)
    x = ht.random.randn(20000, 12)
    y = ht.matmul(x, ht.random.randn(12, 1)) + 0.05 * ht.random.randn(20000, 1)
    res = []
    monkeypatch.setenv("HEAT_LASSO_SOLVER", "sweep")
    for flag in ("0", "1"):
        monkeypatch.setenv("HEAT_AMD_NO_GRAPHS", flag)
        est = ht.regression.Lasso(lam=0.01, max_iter=20, tol=None)
        est.fit(x, y)
        res.append(est.theta.larray.clone())
    assert torch.equal(res[0], res[1]), (res[0] - res[1]).abs().max()


@pytest.mark.parametrize("n", [12, 90])
def test_lasso_sweep_bit_reproducible(gpu, monkeypatch, n):
    """The sweep solver's dot products and column norms are summed in a fixed order (per-workgroup
    slots, last-arriving block / one workgroup per column): repeated fits give identical bits."""
    import heat_amd as ht
    from heat_amd import ops

    ht.random.seed(9)
    x = ht.random.randn(300_001, n)
    y = ht.matmul(x, ht.random.randn(n, 1)) + 0.05 * ht.random.randn(300_001, 1)
    monkeypatch.setenv("HEAT_LASSO_SOLVER", "sweep")
    res = []
    for _ in range(3):
        est = ht.regression.Lasso(lam=0.01, max_iter=5, tol=None)
        est.fit(x, y)
        res.append(est.theta.larray.clone())
    assert torch.equal(res[0], res[1]) and torch.equal(res[1], res[2])
    XT, colsq = ops.lasso_prepare(x.larray)
    for _ in range(3):
        assert torch.equal(ops.lasso_prepare(x.larray)[1], colsq)


@pytest.mark.parametrize("m,k,n", [(300, 257, 129), (1024, 512, 768), (4099, 130, 65), (64, 4096, 64),
                                   (2048, 2048, 2048)])
@pytest.mark.parametrize("layout", ["nn", "tn", "nt", "tt"])
@pytest.mark.parametrize("scale", ["unit", "rows", "tiny", "huge"])
def test_gemm_f16x3(m, k, n, layout, scale):
    """fp16x3 split GEMM within fp32-GEMM error of the fp64 product, for every operand memory order
    and for rows/columns spanning many orders of magnitude."""
    from heat_amd import ops

    dev = _dev()
    g = torch.Generator(device="cpu").manual_seed(m + k + n)
    A = torch.randn(m, k, generator=g)
    B = torch.randn(k, n, generator=g)
    if scale == "rows":      # per-row / per-column magnitudes over 2^-40 .. 2^40, plus zero rows/cols
        A *= torch.pow(2.0, torch.randint(-40, 40, (m, 1), generator=g).float())
        B *= torch.pow(2.0, torch.randint(-40, 40, (1, n), generator=g).float())
        A[::17] = 0
        B[:, ::13] = 0
    elif scale == "tiny":
        A *= 1e-20
        B *= 1e-10
    elif scale == "huge":
        A *= 1e18
        B *= 1e15
    A, B = A.to(dev), B.to(dev)
    if layout[0] == "t":
        A = A.t().contiguous().t()
    if layout[1] == "t":
        B = B.t().contiguous().t()
    C = ops.gemm_f16x3(A, B)
    assert C.dtype == torch.float32 and C.shape == (m, n)
    ref = A.double() @ B.double()
    # split error (<= 2^-21 per product) + fp32 accumulation over the tripled contraction (3k u)
    bound = (A.double().abs() @ B.double().abs()) * (2.0 ** -20 + 3 * k * 2.0 ** -24) + 1e-300
    err = (C.double() - ref).abs()
    assert torch.all(err <= bound), (err / bound).max()
    # same error class as the library fp32 GEMM
    e32 = ((A @ B).double() - ref).abs().max()
    if scale == "unit":
        assert err.max() <= 8 * e32 + 1e-6


def test_gemm_f16x3_nonfinite_falls_back(gpu):
    from heat_amd import ops

    A = torch.randn(256, 128, device="cuda")
    B = torch.randn(128, 64, device="cuda")
    A[3, 5] = float("nan")
    B[7, 9] = float("inf")
    C = ops.gemm_f16x3(A, B)
    ref = A @ B
    assert torch.equal(torch.isnan(C), torch.isnan(ref))
    assert torch.allclose(C[~torch.isnan(ref)], ref[~torch.isnan(ref)], rtol=1e-5, atol=1e-4)


def test_matmul_split_precision(gpu):
    """ht.matmul / ht.linalg.qr honour torch's float32 matmul precision ("high" -> the fused
    fp16x3 kernel gemm_h3t, "highest" -> the exact f32 MFMA kernel), both hand-written for products
    with enough output tiles to fill the GPU (smaller ones go to the library with exact fp32
    products, see test_matmul_small_products_use_library)."""
    import heat_amd as ht
    from heat_amd import ops

    ht.random.seed(2)
    a = ht.random.randn(16384, 1024, split=0)
    b = ht.random.randn(1024, 4096)          # 64 x 16 = 1024 output tiles of 256 x 256
    ref = a.larray.double() @ b.larray.double()
    old = torch.get_float32_matmul_precision()
    calls = []
    orig_h3, orig_f32 = ops.gemm_h3, ops.gemm_f32

    def spy_h3(*args, **kw):
        calls.append("h3")
        return orig_h3(*args, **kw)

    def spy_f32(*args, **kw):
        calls.append("f32")
        return orig_f32(*args, **kw)

    ops.gemm_h3, ops.gemm_f32 = spy_h3, spy_f32
    try:
        torch.set_float32_matmul_precision("high")
        c = ht.matmul(a, b).larray
        q, r = ht.linalg.qr(a)
        assert "h3" in calls and "f32" not in calls, calls
        calls.clear()
        torch.set_float32_matmul_precision("highest")
        c2 = ht.matmul(a, b).larray
        assert calls == ["f32"], calls
    finally:
        torch.set_float32_matmul_precision(old)
        ops.gemm_h3, ops.gemm_f32 = orig_h3, orig_f32
    assert torch.allclose(c2.double(), ref, rtol=1e-5, atol=1e-3)
    assert torch.allclose(c.double(), ref, rtol=1e-5, atol=1e-3)
    qr = q.larray.double() @ r.larray.double()
    assert torch.allclose(qr, a.larray.double(), atol=1e-4)
    qd = q.larray.double()
    assert torch.allclose(qd.T @ qd, torch.eye(qd.shape[1], dtype=torch.float64, device="cuda"), atol=1e-4)


def test_matmul_small_products_use_library(gpu):
    """A product whose 256-tiles cannot fill the CUs runs on the library with EXACT fp32 products
    under either precision setting (no hand-written kernel is called) and matches fp64."""
    import heat_amd as ht
    from heat_amd import ops

    ht.random.seed(5)
    a = ht.random.randn(2048, 1024, split=0)
    b = ht.random.randn(1024, 2048)
    ref = a.larray.double() @ b.larray.double()
    calls = []
    orig_h3, orig_f32 = ops.gemm_h3, ops.gemm_f32
    ops.gemm_h3 = lambda *x, **k: calls.append("h3") or orig_h3(*x, **k)
    ops.gemm_f32 = lambda *x, **k: calls.append("f32") or orig_f32(*x, **k)
    old = torch.get_float32_matmul_precision()
    try:
        for prec in ("high", "highest"):
            torch.set_float32_matmul_precision(prec)
            c = ht.matmul(a, b).larray
            assert torch.get_float32_matmul_precision() == prec
            err = ((c.double() - ref).abs() / (a.larray.abs().double() @ b.larray.abs().double())).max().item()
            assert err < 1024 * 2.0 ** -24, (prec, err)   # exact-fp32 class, not a reduced-precision path
    finally:
        torch.set_float32_matmul_precision(old)
        ops.gemm_h3, ops.gemm_f32 = orig_h3, orig_f32
    assert calls == [], calls


@pytest.mark.parametrize("m,n", [(5000, 300), (131, 64), (20000, 1024)])
def test_gemm_f16x3_gram(m, n):
    """X^T X from one shared split (the QR / Gram path) == the generic split GEMM == fp64."""
    from heat_amd import ops

    dev = _dev()
    g = torch.Generator(device="cpu").manual_seed(m)
    X = (torch.randn(m, n, generator=g) * torch.pow(2.0, torch.randint(-20, 20, (1, n), generator=g).float())).to(dev)
    assert ops.kernels._is_gram(X.t(), X)
    G = ops.gemm_f16x3(X.t(), X)
    ref = X.double().t() @ X.double()
    bound = (X.double().abs().t() @ X.double().abs()) * (2.0 ** -20 + 3 * m * 2.0 ** -24)
    err = (G.double() - ref).abs()
    assert torch.all(err <= bound)
    # relative to the diagonal (no cancellation): same error class as the library fp32 GEMM
    d = ref.diagonal()
    e32 = (((X.t() @ X).double() - ref).abs().diagonal() / d).max()
    assert (err.diagonal() / d).max() <= 8 * e32 + 1e-7


@pytest.mark.parametrize("nq,nt,f", [(1000, 5000, 3), (777, 300, 18), (4096, 20000, 64), (300, 1000, 100),
                                     (513, 129, 128), (50, 7, 16)])
@pytest.mark.parametrize("k", [1, 5, 8, 16])
def test_knn_topk(nq, nt, f, k):
    """Fused distance + running top-k kernel == exact fp64 k nearest neighbours (up to near-ties)."""
    from heat_amd import ops

    dev = _dev()
    g = torch.Generator(device="cpu").manual_seed(nq + nt + f + k)
    Q = torch.randn(nq, f, generator=g).to(dev)
    T = torch.randn(nt, f, generator=g).to(dev)
    dist, idx = ops.knn_topk(Q, T, k)
    assert dist.shape == (nq, k) and idx.dtype == torch.int64
    d = torch.cdist(Q.double(), T.double()) ** 2
    kk = min(k, nt)
    ref, _ = torch.topk(d, kk, dim=1, largest=False)
    assert torch.allclose(dist[:, :kk].double(), ref, rtol=1e-5, atol=1e-5)
    # the reported indices really are at the reported distances
    assert torch.allclose(d.gather(1, idx[:, :kk]), dist[:, :kk].double(), rtol=1e-5, atol=1e-5)
    if kk < k:
        assert torch.all(idx[:, kk:] == -1) and torch.all(torch.isinf(dist[:, kk:]))
    # the kernel's own (quadratic-expansion) distances, which also rank the split partial lists
    draw, _ = ops.knn_topk(Q, T, k, exact_distances=False)
    scale = (Q.double() ** 2).sum(1, keepdim=True) + (T.double() ** 2).sum(1).max()
    assert torch.all((draw[:, :kk].double() - ref).abs() <= 1e-5 * scale)
    # no duplicate neighbours
    s, _ = idx[:, :kk].sort(1)
    assert torch.all(s[:, 1:] != s[:, :-1])


def test_knn_classifier_fused(gpu):
    import heat_amd as ht

    ht.random.seed(4)
    X = ht.random.randn(3000, 8, split=0)
    y = (X.larray[:, 0] > 0).long()
    yd = ht.array(y, is_split=0)
    knn = ht.classification.KNeighborsClassifier(n_neighbors=5)
    knn.fit(X, yd)
    pred = knn.predict(X[:500]).larray
    Xd = X.larray.double()
    d = torch.cdist(Xd[:500], Xd)
    nn_idx = d.topk(5, largest=False).indices
    ref = (y[nn_idx].sum(1) >= 3).long()
    assert (pred.cpu() == ref.cpu()).float().mean() > 0.99


@pytest.mark.parametrize("n,f", [(1000, 3), (70001, 64), (5000, 18), (3000, 128), (777, 200), (100, 1), (300000, 60),
                                 (384, 64), (100, 64), (129, 64)])
@pytest.mark.parametrize("k", [1, 3, 8, 16])
def test_kmeans_step_small(n, f, k):
    """Fused small-k Lloyd pass: labels == fp64 argmin, sums/counts == index_add of the points."""
    from heat_amd import ops

    dev = _dev()
    g = torch.Generator(device="cpu").manual_seed(n * 3 + k + f)
    X = torch.randn(n, f + 3, generator=g).to(dev)[:, :f]   # strided rows
    for Xv in (X, X.contiguous()):
        C = torch.randn(k, f, generator=g).to(dev)
        res = ops.kmeans_step_small(Xv, C)
        if f > 64:
            assert res is None
            continue
        lab, sums, counts = res
        d = torch.cdist(Xv.double(), C.double()) ** 2
        chosen = d.gather(1, lab.long().unsqueeze(1)).squeeze(1)
        assert torch.all(chosen - d.min(1).values <= 1e-5 * (1 + d.min(1).values))
        ref = torch.zeros(k, f, dtype=torch.float64, device=dev).index_add_(0, lab.long(), Xv.double())
        mag = torch.zeros(k, f, dtype=torch.float64, device=dev).index_add_(0, lab.long(), Xv.double().abs())
        assert torch.all((sums.double() - ref).abs() <= 1e-6 * mag + 1e-6)
        assert torch.equal(counts.long(), torch.bincount(lab.long(), minlength=k))


@pytest.mark.parametrize("n,f", [(1000, 3), (70001, 64), (5000, 18), (129, 64), (100000, 64), (64, 64), (65, 64), (127, 64)])
@pytest.mark.parametrize("k", [1, 3, 8, 16])
def test_kmeans_lloyd_small(n, f, k):
    """One-launch-epilogue Lloyd step: new centroids == fp64 means of the assigned points (an empty
    cluster keeps its centroid), shift == sum of squared moves, labels == fp64 argmin; chained calls
    reuse the padded centroids the previous epilogue wrote, and an in-place change of C or a new
    tensor is noticed."""
    from heat_amd import ops

    dev = _dev()
    g = torch.Generator(device="cpu").manual_seed(n + 7 * k + f)
    X = torch.randn(n, f, generator=g).to(dev)
    C = torch.randn(k, f, generator=g).to(dev)
    if k > 1:
        C[-1] = 1e4   # far away: empty cluster
    for it in range(4):
        lab, newC, shift = ops.kmeans_lloyd_small(X, C)
        d = torch.cdist(X.double(), C.double()) ** 2
        chosen = d.gather(1, lab.long().unsqueeze(1)).squeeze(1)
        assert torch.all(chosen - d.min(1).values <= 1e-5 * (1 + d.min(1).values))
        cnt = torch.bincount(lab.long(), minlength=k).double()
        sums = torch.zeros(k, f, dtype=torch.float64, device=dev).index_add_(0, lab.long(), X.double())
        ref = torch.where(cnt.unsqueeze(1) > 0, sums / cnt.clamp(min=1).unsqueeze(1), C.double())
        assert torch.allclose(newC.double(), ref, rtol=1e-5, atol=1e-6)
        if k > 1:
            assert torch.equal(newC[-1], C[-1])
        assert abs(float(shift) - float(((newC.double() - C.double()) ** 2).sum())) <= 1e-6 * (1 + float(shift))
        if it == 1:
            newC.mul_(0.5)          # in place: the padded copy is stale, must be rebuilt
        elif it == 2:
            newC = newC.clone()     # another tensor with the same values
        C = newC


@pytest.mark.parametrize("n,f", [(1000, 3), (70001, 64), (5000, 18), (3000, 128), (777, 200)])
@pytest.mark.parametrize("k", [1, 3, 8, 16])
def test_kmeans_assign_small_k(n, f, k):
    """k <= 16: exact VALU kernel, labels == fp64 argmin (ties -> lowest index), exact min distance."""
    from heat_amd import ops

    dev = _dev()
    g = torch.Generator(device="cpu").manual_seed(n + k + f)
    X = torch.randn(n, f, generator=g).to(dev)
    C = torch.randn(k, f, generator=g).to(dev)
    if k > 1:
        C[-1] = C[0]          # exact duplicate centroid: never chosen over index 0
    lab, mind = ops.kmeans_assign(X, C)
    d = torch.cdist(X.double(), C.double()) ** 2
    ref_min, ref_lab = d.min(1)
    chosen = d.gather(1, lab.long().unsqueeze(1)).squeeze(1)
    assert torch.all(chosen - ref_min <= 1e-5 * (1 + ref_min))
    assert (lab.long() == ref_lab).float().mean() > 0.9999
    if k > 1:
        assert not torch.any(lab == k - 1)
    assert torch.allclose(mind.double(), ref_min, rtol=1e-5, atol=1e-5)
    Xs = X[:, : max(1, f - 1)]   # strided rows (no 16-byte alignment): scalar path
    lab2, _ = ops.kmeans_assign(Xs, C[:, : Xs.shape[1]].contiguous())
    d2 = torch.cdist(Xs.double(), C[:, : Xs.shape[1]].double()) ** 2
    assert (lab2.long() == d2.argmin(1)).float().mean() > 0.9999


@pytest.mark.parametrize("c,k", [(1, 1), (5, 3), (16, 8), (32, 8), (32, 32), (20, 16)])
@pytest.mark.parametrize("f", [1, 3, 18, 128])
@pytest.mark.parametrize("idx64", [False, True])
def test_knn_rescore_kernel(c, k, f, idx64):
    """Fused exact rescoring of candidate lists (csrc/knn_rescore.hip) == the torch formulation:
    difference-form fp32 distances, k smallest in (distance, index) order, -1 candidates ignored,
    duplicate rows (equal distances) ordered by index; strided / unaligned query rows."""
    from heat_amd.ops import kernels as K

    dev = _dev()
    g = torch.Generator(device="cpu").manual_seed(c * 100 + k + f)
    nq, nt = 3001, 500
    T = torch.randn(nt, f, generator=g).to(dev)
    T[100:120] = T[:20]                                     # equal distances at different indices
    Qw = torch.randn(nq, f + 1, generator=g).to(dev)
    cand = torch.randint(0, nt, (nq, c), generator=g)
    cand[::7, -1] = -1                                      # missing candidates
    if c >= 2:
        cand[::5, 0] = cand[::5, 0] % 20                    # rows i and i + 100 hold the same values
        cand[::5, 1] = cand[::5, 0] + 100
    cand = cand.to(dev).to(torch.int64 if idx64 else torch.int32)
    for Q in (Qw[:, :f], Qw[:, :f].contiguous()):
        d, i = K._knn_exact_select(Q, T, cand, k)
        assert d.shape == (nq, k) and i.dtype == torch.int64
        # torch reference of the same semantics
        ci = cand.long()
        nb = T[ci.clamp(min=0)]
        rd = ((Q.unsqueeze(1) - nb) ** 2).sum(-1)
        rd = torch.where(ci >= 0, rd, torch.full_like(rd, float("inf")))
        key_d = torch.sort(rd, dim=1).values
        assert torch.allclose(d.double(), key_d[:, :k].double(), rtol=1e-5, atol=1e-6)
        valid = i >= 0
        # every reported index is one of the query's candidates at the reported distance
        hit = (ci.unsqueeze(2) == i.unsqueeze(1)) & valid.unsqueeze(1)
        assert torch.all(hit.any(1) | ~valid)
        dd = ((Q.unsqueeze(1) - T[i.clamp(min=0)]) ** 2).sum(-1)
        assert torch.allclose(torch.where(valid, dd, d), d, rtol=1e-5, atol=1e-6)
        # ordering: ascending distance, ascending index among equal distances, -1 only after the rest
        nxt_d, prv_d = d[:, 1:], d[:, :-1]
        assert torch.all(nxt_d >= prv_d)
        eq = (nxt_d == prv_d) & valid[:, 1:] & valid[:, :-1]
        assert torch.all(i[:, 1:][eq] >= i[:, :-1][eq])   # (randint may repeat a candidate)
        nvalid = (ci >= 0).sum(1).clamp(max=k)
        assert torch.equal(valid.sum(1), nvalid)


@pytest.mark.parametrize("f,k", [(128, 8), (64, 8), (18, 8), (16, 1), (128, 4)])
def test_knn_certified_one_term(f, k):
    """The certified one-term pass (h1_topk: 16 candidates per query from hi.hi scores + a rigorous
    bound, uncertain queries re-run through the 3-term kernel, exact rescoring) gives the exact
    fp64 k nearest neighbours, including on duplicated training rows (exact ties: the uncertain
    path must run) and near-duplicate queries."""
    from heat_amd import ops
    from heat_amd.ops import kernels as K

    dev = _dev()
    g = torch.Generator(device="cpu").manual_seed(f)
    nq, nt = 140_000, 20_000                # enough query blocks for the single-split path
    Q = torch.randn(nq, f, generator=g).to(dev)
    T = torch.randn(nt, f, generator=g).to(dev)
    T[:600] = T[600:1200]                                   # exact duplicates -> ties
    Q[:3000] = T[:3000] + 1e-3 * torch.randn(3000, f, generator=g).to(dev)
    # 40 training rows of exactly equal norm (sign flips of one vector) nearest to 100 zero queries:
    # more exact ties than candidates (16 or 32), so those queries cannot be certified and take the
    # 3-term path
    base = 0.05 * torch.randn(f, generator=g)
    flips = torch.where(torch.rand(40, f, generator=g) < 0.5, -1.0, 1.0)
    T[1200:1240] = (flips * base).to(dev)
    Q[3000:3100] = 0.0
    before = dict(K._KNN_STATS)
    dist, idx = ops.knn_topk(Q, T, k)
    assert K._KNN_STATS["queries"] - before["queries"] == nq          # the certified path ran
    rechecked = K._KNN_STATS["rechecked"] - before["rechecked"]
    assert 100 <= rechecked < nq // 2, rechecked
    sel = torch.cat([torch.arange(3100), torch.randint(3100, nq, (3000,), generator=g)]).to(dev)
    d = torch.cdist(Q[sel].double(), T.double()) ** 2
    # reference order: distance, then index (stable sort over ascending indices)
    rd, ri = torch.sort(d, dim=1, stable=True)
    rd, ri = rd[:, :k], ri[:, :k]
    assert torch.allclose(dist[sel].double(), rd, rtol=1e-5, atol=1e-5)
    # the reported indices sit at the reported distances; index sets equal wherever the k-th
    # distance is not tied with the (k+1)-th
    assert torch.allclose(d.gather(1, idx[sel]), dist[sel].double(), rtol=1e-5, atol=1e-5)
    clear = (torch.sort(d, dim=1).values[:, k] - rd[:, -1]) > 1e-4 * rd[:, -1].clamp(min=1)
    same = (torch.sort(idx[sel], 1).values == torch.sort(ri, 1).values).all(1)
    assert bool(same[clear].all()), int((~same[clear]).sum())


def test_knn_certified_heterogeneous_norms():
    """Training rows whose norms span 1e-3..1e3 (the certified pass scales all of them by ONE power
    of two, so small rows sit in fp16's subnormal range): the result is still the exact fp64 k
    nearest neighbours - whatever the one-term pass cannot certify goes through the 3-term kernel."""
    from heat_amd import ops
    from heat_amd.ops import kernels as K

    dev = _dev()
    g = torch.Generator(device="cpu").manual_seed(11)
    nq, nt, f, k = 140_000, 9_000, 40, 5
    T = torch.randn(nt, f, generator=g) * torch.pow(10.0, torch.empty(nt, 1).uniform_(-3, 3, generator=g))
    Q = T[torch.randint(0, nt, (nq,), generator=g)] * (1 + 1e-2 * torch.randn(nq, 1, generator=g))
    Q, T = Q.to(dev), T.to(dev)
    before = dict(K._KNN_STATS)
    dist, idx = ops.knn_topk(Q, T, k)
    assert K._KNN_STATS["queries"] - before["queries"] == nq
    sel = torch.randint(0, nq, (4000,), generator=g).to(dev)
    d = torch.cdist(Q[sel].double(), T.double()) ** 2
    rd, ri = torch.sort(d, dim=1, stable=True)
    rd = rd[:, :k]
    assert torch.allclose(dist[sel].double(), rd, rtol=1e-4, atol=1e-6)
    assert torch.allclose(d.gather(1, idx[sel]), rd, rtol=1e-4, atol=1e-6)


@pytest.mark.parametrize("metric", ["euclidean", "sqeuclidean", "gaussian", "manhattan"])
@pytest.mark.parametrize("n,f", [(1000, 18), (129, 3), (257, 40), (4000, 64), (1, 5)])
def test_cdist_symmetric_compute_once(metric, n, f):
    """Y is X on the difference kernels: upper-triangle tiles + mirrored stores give the same
    matrix as the full launch, exactly symmetric, with an exact zero diagonal."""
    from heat_amd import ops

    dev = _dev()
    g = torch.Generator(device="cpu").manual_seed(n + f)
    X = torch.rand(n, f, generator=g).to(dev)
    full = ops.cdist(X, X.clone(), metric, sigma=1.5, exact=True)
    sym = ops.cdist(X, X, metric, sigma=1.5, exact=True, symmetric=True)
    assert torch.equal(sym, sym.t())
    assert torch.allclose(sym, full, rtol=1e-6, atol=1e-6)
    if metric != "gaussian":
        assert torch.all(torch.diagonal(sym) == 0)
    big = torch.full((n, n + 5), -1.0, device=dev)
    ops.cdist(X, X, metric, sigma=1.5, exact=True, symmetric=True, out=big[:, :n])
    assert torch.equal(big[:, :n], sym) and torch.all(big[:, n:] == -1.0)
