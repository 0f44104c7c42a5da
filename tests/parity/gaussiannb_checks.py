"""Parity with ``heat/naive_bayes/tests/test_gaussiannb.py``: fits the reference's iris train/test
split (plain CSV fixtures) and compares class priors, epsilon, theta, sigma and predict_proba with
the scikit-learn values the reference stores (``iris_y_pred_proba.csv``), replicated and split,
with and without sample weights, plus partial_fit and the ValueErrors."""
import os

import numpy as np
import torch

import heat_amd as ht

from ._util import close, raises, same

DS = "/root/reference/heat/datasets"
PRIOR = np.array([0.38666667, 0.26666667, 0.34666667])
THETA = np.array([[4.97586207, 3.35862069, 1.44827586, 0.23448276], [5.935, 2.71, 4.185, 1.3],
                  [6.77692308, 3.09230769, 5.73461538, 2.10769231]])
SIGMA = np.array([[0.10321047, 0.13208086, 0.01629013, 0.00846612], [0.256275, 0.0829, 0.255275, 0.046],
                  [0.38869823, 0.10147929, 0.31303255, 0.04763314]])


def _data(split=None):
    ld = lambda n, dt: ht.load(os.path.join(DS, n), sep=";", dtype=dt, split=split)  # noqa: E731
    return (ld("iris_X_train.csv", ht.float64), ld("iris_X_test.csv", ht.float64),
            ld("iris_y_train.csv", ht.int64).squeeze(), ld("iris_y_test.csv", ht.int64).squeeze(),
            ht.load(os.path.join(DS, "iris_y_pred_proba.csv"), sep=";", dtype=ht.float64))


def test_classifier():
    g = ht.naive_bayes.GaussianNB()
    assert ht.is_estimator(g) and ht.is_classifier(g)


def test_get_and_set_params():
    g = ht.naive_bayes.GaussianNB()
    params = g.get_params()
    assert params == {"priors": None, "var_smoothing": 1e-9}
    params["var_smoothing"] = 1e-10
    g.set_params(**params)
    assert g.var_smoothing == 1e-10


def test_fit_iris():
    if not os.path.exists(os.path.join(DS, "iris_X_train.csv")):
        return
    for split in (None, 0):
        X_train, X_test, y_train, y_test, proba_sk = _data(split)
        g = ht.naive_bayes.GaussianNB()
        assert g.priors is None
        for attr in ("classes_", "class_prior_", "epsilon_"):
            try:
                getattr(g, attr)
                raise AssertionError("{} before fit".format(attr))
            except AttributeError:
                pass
        fit = g.fit(X_train, y_train)
        same(g.classes_, np.array([0, 1, 2]))
        y_pred = g.partial_fit(X_train, y_train, classes=None).predict(X_test)
        proba = fit.predict_proba(X_test)
        assert isinstance(y_pred, ht.DNDarray)
        assert int((y_pred != y_test).sum().item()) == 4
        close(g.class_prior_, PRIOR, rtol=1e-6)
        close(g.epsilon_, np.array([3.6399040000000003e-09]), rtol=1e-6)
        # theta/sigma after fit + partial_fit with the same data (counts doubled, moments equal)
        close(g.theta_, THETA, rtol=1e-6, atol=1e-6)
        close(g.sigma_, SIGMA, atol=1e-6)
        close(proba, proba_sk.numpy(), atol=1e-6)
        w = ht.ones(y_train.gshape[0], dtype=ht.float32, split=split)
        fw = g.fit(X_train, y_train, sample_weight=w)
        close(g.class_prior_, PRIOR, rtol=1e-6)
        close(g.theta_, THETA, rtol=1e-6, atol=1e-6)
        same(fw.predict(X_test), y_pred.numpy())
        close(fw.predict_proba(X_test), proba_sk.numpy(), atol=1e-6)
    X_train, X_test, y_train, y_test, _ = _data()
    g = ht.naive_bayes.GaussianNB()
    raises(ValueError, g.fit, torch.ones(3, 4), y_train)
    raises(ValueError, g.fit, X_train, np.ones(75))
    raises(ValueError, g.fit, X_train, ht.ones((75, 2)))
    raises(ValueError, g.fit, X_train, y_train, sample_weight=torch.ones(75))
    raises(ValueError, g.fit, ht.ones((75, 4, 2)), y_train)
    raises(ValueError, g.fit, X_train, ht.ones(74, dtype=ht.int64))
    g.fit(X_train, y_train)
    raises(ValueError, g.predict, torch.ones(3, 4))
    raises(ValueError, g.partial_fit, ht.ones((75, 5)), y_train)
    raises(ValueError, g.partial_fit, X_train, y_train, classes=ht.array([0, 1, 7]))
    raises(ValueError, g.fit, X_train, y_train, sample_weight=ht.ones((75, 2)))
    raises(ValueError, g.fit, X_train, y_train, sample_weight=ht.ones(74))
    for pr in (ht.array([0.5, 0.5]), ht.array([0.5, 0.4, 0.3]), ht.array([1.2, -0.1, -0.1])):
        g2 = ht.naive_bayes.GaussianNB(priors=pr)
        raises(ValueError, g2.fit, X_train, y_train)
