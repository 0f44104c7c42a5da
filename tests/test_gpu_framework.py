"""The whole CPU check suite again with the default device on the MI355X (world of one): every
factory, op, estimator and I/O path must keep its tensors on the GPU and agree with NumPy."""
import pytest

from . import dist_checks

pytestmark = pytest.mark.gpu

CHECKS = [n for n in dir(dist_checks) if n.startswith("check_")]


@pytest.mark.parametrize("name", CHECKS)
def test_on_gpu(name, gpu):
    getattr(dist_checks, name)()


def test_lasso_kernel_matches_host(gpu):
    import numpy as np
    import torch
    import heat_amd as ht

    rng = np.random.default_rng(0)
    X = rng.normal(size=(5000, 40)).astype(np.float32)
    X /= np.sqrt((X ** 2).mean(0))
    y = (X @ rng.normal(size=40).astype(np.float32)).astype(np.float32)
    th = []
    for dev in ("cpu", "gpu"):
        est = ht.regression.Lasso(lam=0.05, max_iter=30, tol=None)
        est.fit(ht.array(X, device=dev), ht.array(y[:, None], device=dev))
        th.append(est.theta.larray.cpu())
    assert torch.allclose(th[0], th[1], atol=2e-4), (th[0] - th[1]).abs().max()


def test_profiling_counts_native_kernels(gpu):
    import torch
    import heat_amd as ht
    from heat_amd import profiling

    profiling.reset()
    profiling.enable(timing=True)
    try:
        x = ht.random.randn(4096, 16, split=0)
        km = ht.cluster.KMeans(n_clusters=8, init="random", max_iter=3)
        km.fit(x)
        c = profiling.counters()
    finally:
        profiling.disable()
    assert c["kmeans_assign"]["calls"] >= 3 and c["kmeans_assign"]["ms"] > 0
