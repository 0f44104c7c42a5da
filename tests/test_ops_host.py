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
