"""Parity with ``heat/cluster/tests/test_spectral.py``: estimator traits and parameters, iris fits
with the fully-connected and epsilon-neighbour Laplacians (rbf / euclidean), kmeans params passed
through, and the errors. Labels must separate the setosa class."""
import numpy as np

import heat_amd as ht

from ._ml import iris
from ._util import raises


def test_clusterer():
    s = ht.cluster.Spectral()
    assert ht.is_estimator(s) and ht.is_clusterer(s)


def test_get_and_set_params():
    s = ht.cluster.Spectral()
    params = s.get_params()
    assert params == {"n_clusters": None, "gamma": 1.0, "metric": "rbf", "laplacian": "fully_connected",
                      "threshold": 1.0, "boundary": "upper", "n_lanczos": 300, "assign_labels": "kmeans"}, params
    params["n_clusters"] = 10
    s.set_params(**params)
    assert s.n_clusters == 10


def test_fit_iris():
    x = iris(0)
    m = 10
    s = ht.cluster.Spectral(n_clusters=3, gamma=1.0, metric="rbf", laplacian="fully_connected", n_lanczos=m)
    s.fit(x)
    assert isinstance(s.labels_, ht.DNDarray) and s.labels_.shape[0] == 150
    lab = s.labels_.numpy().reshape(-1)
    assert len(set(lab[:50].tolist())) == 1 and lab[0] not in set(lab[50:].tolist())
    labels = ht.cluster.Spectral(metric="euclidean", laplacian="eNeighbour", threshold=0.5, boundary="upper",
                                 n_lanczos=m).fit_predict(x)
    assert isinstance(labels, ht.DNDarray)
    labels = ht.cluster.Spectral(gamma=0.1, metric="rbf", laplacian="eNeighbour", threshold=0.5, boundary="upper",
                                 n_lanczos=m).fit_predict(x)
    assert isinstance(labels, ht.DNDarray)
    kmeans = {"kmeans++": "kmeans++", "max_iter": 30, "tol": -1}
    labels = ht.cluster.Spectral(n_clusters=3, gamma=1.0, normalize=True, n_lanczos=m, params=kmeans).fit_predict(x)
    assert isinstance(labels, ht.DNDarray)
    raises(NotImplementedError, ht.cluster.Spectral, metric="ahalanobis", n_lanczos=m)
    raises(NotImplementedError, ht.cluster.Spectral(n_lanczos=20).fit, iris(1))
