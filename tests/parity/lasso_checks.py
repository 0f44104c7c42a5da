"""Parity with ``heat/regression/tests/test_lasso.py``: estimator traits/parameters, a 100-sweep
fit on the reference's diabetes fixture (``diabetes.h5``) with attribute shapes, coefficients
against a NumPy coordinate-descent reference of the same update rule, and the errors."""
import os

import numpy as np

import heat_amd as ht

from ._util import close, raises

H5 = "/root/reference/heat/datasets/diabetes.h5"


def test_regressor():
    l = ht.regression.Lasso()
    assert ht.is_estimator(l) and ht.is_regressor(l)


def test_get_and_set_params():
    l = ht.regression.Lasso()
    params = l.get_params()
    assert params == {"lam": 0.1, "max_iter": 100, "tol": 1e-6}
    params["max_iter"] = 200
    l.set_params(**params)
    assert l.max_iter == 200


def test_exceptions():
    raises(ValueError, ht.regression.Lasso().set_params, foo="bar")


def _np_lasso(X, y, lam, iters):
    m, n = X.shape
    th = np.zeros(n)
    for _ in range(iters):
        for j in range(n):
            r = y - X @ th + X[:, j] * th[j]
            rho = X[:, j] @ r / m
            z = X[:, j] @ X[:, j] / m
            if j == 0:
                th[j] = rho / z
            else:
                th[j] = np.sign(rho) * max(abs(rho) - lam, 0.0) / z
    return th


def test_lasso():
    if not os.path.exists(H5):
        return
    for split in (None, 0):
        X = ht.load_hdf5(H5, dataset="x", split=split)
        y = ht.load_hdf5(H5, dataset="y", split=split)
        X = X / ht.sqrt(ht.mean(X ** 2, axis=0))
        m, n = X.shape
        est = ht.regression.lasso.Lasso(max_iter=100, tol=None)
        assert est.lam == 0.1 and est.theta is None and est.n_iter is None and est.max_iter == 100
        assert est.coef_ is None and est.intercept_ is None
        est.fit(X, y)
        assert isinstance(est.theta, ht.DNDarray) and est.n_iter == 100
        assert est.coef_.shape == (n - 1, 1) and est.intercept_.shape == (1,)
        yest = est.predict(X)
        assert isinstance(yest, ht.DNDarray) and yest.shape == (m, 1)
        ref = _np_lasso(X.numpy().astype(np.float64), y.numpy().astype(np.float64).reshape(-1), 0.1, 100)
        close(est.theta.numpy().reshape(-1), ref, rtol=2e-3, atol=2e-3)
        raises(ValueError, est.fit, X, ht.zeros((3, 3, 3)))
        raises(ValueError, est.fit, ht.zeros((3, 3, 3)), ht.zeros((3, 3)))
