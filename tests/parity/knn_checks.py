"""Parity with ``heat/classification/tests/test_knn.py``: KNeighborsClassifier on the iris fixture
(replicated and split), one-hot labels, the one_hot_encoding utility and the shape errors;
predictions are checked against a NumPy k-NN vote."""
import numpy as np
from scipy.spatial.distance import cdist as sp_cdist

import heat_amd as ht
from heat_amd.classification.kneighborsclassifier import KNeighborsClassifier

from ._ml import iris, iris_labels
from ._util import raises, same


def _np_knn(x, y, q, k):
    d = sp_cdist(q, x)
    idx = np.argsort(d, axis=1, kind="stable")[:, :k]
    votes = y[idx]
    return np.array([np.bincount(v, minlength=3).argmax() for v in votes])


def _case(split):
    x = iris(split)
    y = ht.array(iris_labels(), split=split)
    knn = KNeighborsClassifier(n_neighbors=5)
    knn.fit(x, y)
    r = knn.predict(x)
    assert ht.is_estimator(knn) and ht.is_classifier(knn)
    assert isinstance(r, ht.DNDarray) and r.shape == y.shape
    xn = x.numpy().astype(np.float64)
    ref = _np_knn(xn, iris_labels(), xn, 5)
    agree = (r.numpy().reshape(-1) == ref).mean()
    assert agree > 0.97, agree


def test_split_none():
    _case(None)


def test_split_zero():
    _case(0)


def test_exception():
    a, b, c = ht.zeros((3,)), ht.zeros((3, 2)), ht.zeros((2, 2, 2))
    raises(ValueError, KNeighborsClassifier(n_neighbors=1).fit, a, b)
    raises(ValueError, KNeighborsClassifier(n_neighbors=1).fit, b, c)
    raises(ValueError, KNeighborsClassifier(n_neighbors=1).fit, c, a)


def test_utility():
    one_hot = KNeighborsClassifier.one_hot_encoding(ht.array([1, 2, 3, 4]))
    assert (one_hot == ht.array([[0, 1, 0, 0, 0], [0, 0, 1, 0, 0], [0, 0, 0, 1, 0], [0, 0, 0, 0, 1]])).all()


def test_fit_one_hot():
    x = iris(None)
    labels = ht.array(iris_labels(), split=0)
    one_hot = ht.array(np.eye(3, dtype=np.int64)[iris_labels()], split=0)
    a = KNeighborsClassifier(n_neighbors=5)
    a.fit(x, labels)
    b = KNeighborsClassifier(n_neighbors=5)
    b.fit(x, one_hot)
    ra, rb = a.predict(x), b.predict(x)
    assert ra.shape == labels.shape
    same(rb if rb.ndim == 1 else ht.argmax(rb, axis=1), ra.numpy())
