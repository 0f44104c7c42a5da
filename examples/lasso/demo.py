"""
Lasso demo (reference ``examples/lasso/demo.py``): regularisation path of coordinate-descent
Lasso on the diabetes data (the reference fixture when available, else a synthetic stand-in);
prints the coefficients per lambda.

    python -m heat_amd.run -n 2 examples/lasso/demo.py
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import numpy as np  # noqa: E402

import heat_amd as ht  # noqa: E402


def main():
    X, y = ht.datasets.diabetes(split=0)
    path = []
    for lam in np.logspace(-3, 0.5, 8):
        est = ht.regression.Lasso(lam=float(lam), max_iter=200, tol=1e-6)
        est.fit(X, y)
        theta = est.theta.numpy().ravel()
        path.append(theta)
        rmse = est.rmse(y, est.predict(X))  # collective: every rank calls it
        if ht.MPI_WORLD.rank == 0:
            print("lambda={:8.4f} nonzero={:2d} rmse={:.4f} theta={}".format(
                lam, int((np.abs(theta[1:]) > 0).sum()), rmse, theta.round(3)))


if __name__ == "__main__":
    main()
