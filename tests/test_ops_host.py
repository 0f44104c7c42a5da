"""Host (CPU) behaviour of the native-kernel entry points: the PyTorch reference paths that serve
host tensors and act as the numerics oracle of the GPU tests."""
import torch

from heat_amd import ops
from heat_amd.core.linalg import basics


def test_knn_topk_host_matches_bruteforce():
    g = torch.Generator().manual_seed(0)
    Q = torch.randn(50, 7, generator=g)
    T = torch.randn(300, 7, generator=g)
    d, i = ops.knn_topk(Q, T, 5)
    ref = torch.cdist(Q.double(), T.double()) ** 2
    rv, ri = ref.topk(5, largest=False)
    assert torch.allclose(d.double(), rv, rtol=1e-5, atol=1e-6)
    assert torch.equal(i, ri)
    # fewer training rows than k: padded with +inf / -1
    d, i = ops.knn_topk(Q, T[:3], 5)
    assert torch.all(i[:, 3:] == -1) and torch.all(torch.isinf(d[:, 3:]))


def test_gemm_split_host_is_plain_matmul():
    a, b = torch.randn(40, 30), torch.randn(30, 20)
    assert torch.allclose(ops.gemm_f16x3(a, b), a @ b)
    assert not basics._split_gemm_ok(a, b)   # host tensors never take the device split path


def test_small_k_pass_is_device_only():
    X, C = torch.randn(100, 8), torch.randn(4, 8)
    assert ops.kmeans_step_small(X, C) is None
    lab, mind = ops.kmeans_assign(X, C)
    d = torch.cdist(X.double(), C.double()) ** 2
    assert torch.equal(lab.long(), d.argmin(1))
    assert torch.allclose(mind.double(), d.min(1).values, rtol=1e-5, atol=1e-5)


def test_kmeans_update_host():
    X = torch.randn(500, 6)
    lab = torch.randint(0, 7, (500,), dtype=torch.int32)
    s, c = ops.kmeans_update(X, lab, 7)
    ref = torch.zeros(7, 6, dtype=torch.float64).index_add_(0, lab.long(), X.double())
    assert torch.allclose(s.double(), ref, atol=1e-4)
    assert torch.equal(c.long(), torch.bincount(lab.long(), minlength=7))


def _lasso_reference_loop(X, y, lam, max_iter, tol):
    """The reference's data-form coordinate descent (heat/regression/lasso.py:121-175) in fp64 numpy."""
    import numpy as np

    m, n = X.shape
    th = np.zeros(n)
    it = 0
    for it in range(1, max_iter + 1):
        old_all = th.copy()
        for j in range(n):
            rho = np.mean(X[:, j] * (y - X @ th + th[j] * X[:, j]))
            th[j] = rho if j == 0 else np.sign(rho) * max(abs(rho) - lam, 0.0)
        if tol is not None and np.sqrt(np.mean((th - old_all) ** 2)) < tol:
            break
    return th, it


def test_lasso_gram_cd_host_matches_reference_loop():
    import numpy as np

    rng = np.random.default_rng(1)
    X = rng.normal(size=(800, 9))
    X[:, 0] = 1.0
    X /= np.sqrt((X ** 2).mean(0))
    y = X @ rng.normal(size=9) + 0.1 * rng.normal(size=800)
    G = ops.lasso_gram(torch.from_numpy(X).float(), torch.from_numpy(y).float())
    A = np.concatenate([X.astype(np.float32).astype(np.float64), y.astype(np.float32).astype(np.float64)[:, None]], 1)
    assert torch.allclose(G, torch.from_numpy(A.T @ A), rtol=1e-10)
    G = G / 800
    for tol in (None, 1e-6):
        th = torch.zeros(9, dtype=torch.float64)
        it = ops.lasso_cd(G[:9, :9], G[:9, 9].contiguous(), 0.05, 40, tol, th)
        ref, rit = _lasso_reference_loop(A[:, :9], A[:, 9], 0.05, 40, tol)
        assert it == rit
        assert np.allclose(th.numpy(), ref, atol=1e-9)


def test_lasso_gram_blocked_matches_fp64():
    from heat_amd.ops.kernels import _gram_blocked

    g = torch.Generator().manual_seed(3)
    for m, n in [(3000, 5), (70001, 130)]:
        X, y = torch.randn(m, n, generator=g), torch.randn(m, generator=g)
        A = torch.cat([X, y[:, None]], 1).double()
        ref = A.T @ A
        assert torch.allclose(_gram_blocked(X, y), ref, rtol=0, atol=1e-6 * ref.abs().max().item())


# ---- C ABI workspace contracts of the fused / fixed-order kernels (host functions of the library;
# the GPU tests exercise the kernels that rely on them)
def _lib():
    import pytest

    try:
        return ops.lib()
    except Exception as e:  # pragma: no cover - library not built
        pytest.skip("native library unavailable: {}".format(e))


def _group(n):
    g = 1
    while g * g < n:
        g += 1
    return g


def test_moments_workspace_contracts():
    import ctypes

    L = _lib()
    pd, nc = ctypes.c_int64(), ctypes.c_int64()
    for nrows in (1, 3, 1000):
        for nchunks in (1, 2, 17, 1024, 4096, 65536):
            L.ha_moments_rows_workspace(nrows, nchunks, ctypes.byref(pd), ctypes.byref(nc))
            g = _group(nchunks)
            ngroups = (nchunks + g - 1) // g
            assert g <= 256 and ngroups <= 256          # one partial per thread at each tree level
            if nchunks == 1:
                assert pd.value == nrows * 3 and nc.value == 0
            else:
                assert pd.value == nrows * (nchunks + ngroups) * 3
                assert nc.value == nrows * (ngroups + 1)
    for ncols in (1, 4, 1000, 4097):
        for nchunks in (1, 5, 256, 65535):
            L.ha_moments_cols_workspace(ncols, nchunks, ctypes.byref(pd), ctypes.byref(nc))
            g = _group(nchunks)
            ngroups = (nchunks + g - 1) // g
            extra = ngroups if nchunks > 1 else 0
            assert pd.value == (nchunks + extra) * ncols * 3
            assert nc.value == ((ncols + 255) // 256) * (ngroups + 1)


def test_certified_assignment_list_capacity():
    """Every filter workgroup (256 points) appends to list blockIdx % shards: a list must hold the
    points of ceil(workgroups / shards) workgroups, and all lists together at least n."""
    L = _lib()
    shards = L.ha_h3_amb_shards()
    assert shards >= 1
    for n in (1, 255, 256, 257, 4096, 12_500_000, 100_000_007):
        total = L.ha_h3_amb_rows(n)
        assert total % shards == 0
        cap = total // shards
        wgs = (n + 255) // 256
        assert cap >= -(-wgs // shards) * 256 and total >= n


def test_lasso_scratch_contracts():
    L = _lib()
    for m, n in ((1, 1), (1000, 3), (10_000_000, 16), (4_000_000, 256), (300, 1024)):
        s = L.ha_lasso_prepare_scratch(m, n)
        assert s >= n and s % n == 0                    # whole per-workgroup column partials
        assert s // n <= max(2048, 8 * 256)             # bounded grid, whatever m
    for ncu in (1, 80, 256, 304):
        assert L.ha_lasso_partial_floats(ncu) >= 4 + 4 * ncu   # result, counter, pad, one slot/block


def test_householder_partial_contracts():
    L = _lib()
    nb, copies = L.ha_hh_nb(), L.ha_hh_counters()
    assert L.ha_hh_slen() == copies * 2 * nb
    for m in (1, 31, 32, 33, 1000, 1_250_000, 10**8):
        part = L.ha_hh_part_len(m)
        blocks = part // nb
        assert part % nb == 0 and 1 <= blocks <= max(1, -(-m // 32))
        gb = -(-blocks // copies)                       # blocks per group of the fixed-order tree
        assert -(-blocks // gb) <= copies               # every group has an accumulator copy


def test_stale_library_after_failed_rebuild_warns(tmp_path, monkeypatch):
    """A rebuild that fails while an older library exists loads it with a loud warning that
    names the failing source; HEAT_STRICT_BUILD=1 refuses instead."""
    import os
    import shutil
    import warnings

    import pytest

    from heat_amd.ops import _build

    real = _build.LIBPATH
    if not os.path.exists(real):
        pytest.skip("native library not built")
    libdir = tmp_path / "_lib"
    libdir.mkdir()
    stale = libdir / "libheat_amd_kernels.so"
    shutil.copy(real, stale)
    bad = tmp_path / "broken_kernel.hip"
    bad.write_text("#include <hip/hip_runtime.h>\n__global__ void k() { this is not C++; }\n")
    os.utime(stale, (1, 1))  # older than every source
    monkeypatch.setattr(_build, "LIBDIR", str(libdir))
    monkeypatch.setattr(_build, "LIBPATH", str(stale))
    monkeypatch.setattr(_build, "sources", lambda: [str(bad)])
    monkeypatch.setattr(_build, "headers", lambda: [])
    saved = ops._lib
    monkeypatch.setattr(ops, "_lib", None)
    try:
        with warnings.catch_warnings(record=True) as rec:
            warnings.simplefilter("always")
            handle = ops.lib()
        msgs = [str(w.message) for w in rec if issubclass(w.category, RuntimeWarning)]
        assert handle is not None
        assert any("STALE" in m and "broken_kernel.hip" in m for m in msgs), msgs
        monkeypatch.setattr(ops, "_lib", None)
        monkeypatch.setenv("HEAT_STRICT_BUILD", "1")
        with pytest.raises(RuntimeError, match="broken_kernel.hip"):
            ops.lib()
    finally:
        ops._lib = saved


def test_topk_lex_wide_indices_fall_back_to_stable_sorts():
    """Global indices from 2^32 - 1 up do not fit the packed 32-bit key: the merge falls back to
    two stable sorts and still orders equal distances by index."""
    import torch
    from heat_amd.ops import kernels

    d = torch.tensor([[3.0, 1.0, 1.0, 0.5, 1.0]])
    big = 0xFFFFFFFF + 10
    idx = torch.tensor([[big + 4, big + 3, big + 1, big + 9, big + 2]])
    dv, di = kernels._topk_lex(d, idx, 3, max_index=big + 9)
    assert dv.tolist() == [[0.5, 1.0, 1.0]] and di.tolist() == [[big + 9, big + 1, big + 2]]
    small = idx - big
    dv2, di2 = kernels._topk_lex(d, small, 3, max_index=9)
    assert dv2.tolist() == dv.tolist() and (di2 + big).tolist() == di.tolist()
