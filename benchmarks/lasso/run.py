"""
lasso benchmark (reference ``benchmarks/lasso/heat-gpu.py:23-29``): wall-clock of
``Lasso(max_iter=1, tol=-1.0).fit(x, y)`` = one coordinate-descent sweep. The reference's strong
size is 1e7 rows (eurad); the feature count of that file is not in the repository, so it is a
parameter (default 16).

Same-node comparator (world of one): the reference's ``torch-gpu.py:48-66`` coordinate descent in
plain torch on the same data (``x @ theta`` per coordinate, a host-side soft threshold per
coordinate), ``max_iter`` sweeps - ``reference_torch_s`` / ``speedup``.
"""
import argparse
import os

from benchmarks import common  # noqa: F401
from benchmarks.common import ht, report, setup, timed, torch_reference


def torch_lasso(x, y, lam: float = 0.1, max_iter: int = 1):
    """The reference's torch comparator (``benchmarks/lasso/torch-gpu.py``): cyclic coordinate
    descent with the full prediction ``x @ theta`` recomputed per coordinate, the soft threshold
    decided on the host (one device sync per coordinate), intercept column 0 not regularised."""
    import torch

    n = x.shape[1]
    theta = torch.zeros(n, 1, device=x.device, dtype=x.dtype)
    for _ in range(max_iter):
        for j in range(n):
            y_est = (x @ theta)[:, 0]
            rho = (x[:, j] * (y - y_est + theta[j] * x[:, j])).mean()
            if j == 0:
                theta[j] = rho
            else:
                r = float(rho)
                theta[j] = r + lam if r < -lam else (r - lam if r > lam else 0.0)
    return theta


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--rows", type=int, default=10_000_000)
    p.add_argument("--features", type=int, default=16)
    p.add_argument("--iterations", type=int, default=1)
    p.add_argument("--trials", type=int, default=5)
    p.add_argument("--no-reference", action="store_true", help="skip the torch comparator")
    a = p.parse_args()
    dev = setup()
    ht.random.seed(3)
    x = ht.random.randn(a.rows, a.features, split=0, device=dev)
    w = ht.random.randn(a.features, 1, device=dev)
    y = ht.matmul(x, w) + 0.1 * ht.random.randn(a.rows, 1, split=0, device=dev)

    def fit():
        ht.regression.Lasso(lam=0.1, max_iter=a.iterations, tol=-1.0).fit(x, y)

    t = timed(fit, a.trials)
    ref = None
    if not a.no_reference:
        xl, yl = x.larray, y.larray.reshape(-1)
        ref = torch_reference(lambda: torch_lasso(xl, yl, 0.1, a.iterations), a.trials)
    report("lasso", {"rows": a.rows, "features": a.features, "iterations": a.iterations,
                     "solver": os.environ.get("HEAT_LASSO_SOLVER", "auto")}, t,
           {"GB_per_s": 4.0 * a.rows * a.features * 2 * a.iterations / 1e9}, reference=ref)


if __name__ == "__main__":
    main()
