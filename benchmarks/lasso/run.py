"""
lasso benchmark (reference ``benchmarks/lasso/heat-gpu.py:23-29``): wall-clock of
``Lasso(max_iter=1, tol=-1.0).fit(x, y)`` = one coordinate-descent sweep. The reference's strong
size is 1e7 rows (eurad); the feature count of that file is not in the repository, so it is a
parameter (default 16).
"""
import argparse
import os

from benchmarks import common  # noqa: F401
from benchmarks.common import ht, report, setup, timed


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--rows", type=int, default=10_000_000)
    p.add_argument("--features", type=int, default=16)
    p.add_argument("--iterations", type=int, default=1)
    p.add_argument("--trials", type=int, default=5)
    a = p.parse_args()
    dev = setup()
    ht.random.seed(3)
    x = ht.random.randn(a.rows, a.features, split=0, device=dev)
    w = ht.random.randn(a.features, 1, device=dev)
    y = ht.matmul(x, w) + 0.1 * ht.random.randn(a.rows, 1, split=0, device=dev)

    def fit():
        ht.regression.Lasso(lam=0.1, max_iter=a.iterations, tol=-1.0).fit(x, y)

    t = timed(fit, a.trials)
    report("lasso", {"rows": a.rows, "features": a.features, "iterations": a.iterations,
                     "solver": os.environ.get("HEAT_LASSO_SOLVER", "auto")}, t,
           {"GB_per_s": 4.0 * a.rows * a.features * 2 * a.iterations / 1e9})


if __name__ == "__main__":
    main()
